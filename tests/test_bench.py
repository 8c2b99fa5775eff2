"""bench.py contract tests on CPU (synthetic MI355X sysfs tree).

The driver runs ``python bench.py --gpus N --steps K --warmup W`` (N>1 under
torch.distributed.run, one rank per GPU); rank 0 must print exactly one JSON
line with the contract's fields.  The multi-rank path is exercised with the
gloo backend and world_size 2 on 127.0.0.1.
"""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _json_lines(stdout: str) -> list[dict]:
    return [json.loads(ln) for ln in stdout.splitlines() if ln.startswith("{")]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_single_process_contract():
    cp = subprocess.run([sys.executable, "bench.py", "--steps", "30", "--warmup", "3", "--backend", "synthetic",
                         "--cold-cycles", "2"], capture_output=True, text=True, timeout=300, cwd=str(REPO))
    assert cp.returncode == 0, cp.stderr[-3000:]
    lines = _json_lines(cp.stdout)
    assert len(lines) == 1
    r = lines[0]
    assert REQUIRED <= set(r)
    assert r["metric"].startswith("label-file generation p50 latency")
    assert r["n_gpus"] == 1 and r["steps"] == 30 and r["warmup"] == 3
    assert r["higher_is_better"] is False and r["unit"] == "ms" and r["scaling"] == "weak"
    assert r["labels_ok"] is True, r["label_problems"]
    assert "synthetic" in r["data"]
    assert 0 < r["value"] < 50
    assert {"init", "enumerate", "label", "write"} <= set(r["phases_p50_ms"])
    assert r["extras"]["oneshot_process"]["p50_ms"] > 0
    assert "--backend=auto" in r["extras"]["oneshot_process"]["args"]  # the Job template's backend
    assert r["oneshot_process_p50_ms"] == r["extras"]["oneshot_process"]["p50_ms"]
    assert r["first_cycle_ms"] > 0
    assert r["cold_cycle"]["interval"] == "1s" and r["cold_cycle"]["cycles"] == 2
    assert r["cold_cycle"]["p50_ms"] > 0 and "write" in r["cold_cycle"]["phases_p50_ms"]
    # Attribution and per-cycle records (round 4): the unattributed time, the
    # CPUs of every cycle, and one row per cycle whose phases add up.
    c = r["cold_cycle"]
    assert c["other_p50_ms"] is not None
    assert len(c["cycle_cpus"]) == len(c["totals_ms"]) == len(c["rows_ms"]) == 2
    # A span missing from the cycle shows in both cycles; one preempted
    # between spans (this is a shared VM) in one.  A sanitized daemon is
    # several times slower everywhere.
    if not os.environ.get("GFD_SANITIZED"):
        assert min(row["other"] for row in c["rows_ms"]) < 0.05, c["rows_ms"]
    for row in c["rows_ms"]:
        top = sum(row.get(k, 0) for k in ("submit", "init", "enumerate", "label", "sriov.join", "merge", "log", "write",
                                           "other"))
        assert top <= row["total"] + 0.02, row
    job = r["extras"]["oneshot_process"]
    assert job["runs"] >= 15 and len(job["runs_ms"]) == job["runs"] and job["first_ms"] == job["runs_ms"][0]


@pytest.mark.parametrize("n", [2, 4, 8])
def test_synthetic_scaling_labels(n):
    cp = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "10", "--warmup", "1", "--backend",
                         "synthetic", "--no-extras"], capture_output=True, text=True, timeout=300, cwd=str(REPO))
    assert cp.returncode == 0, cp.stderr[-3000:]
    r = _json_lines(cp.stdout)[0]
    assert r["n_gpus"] == n and r["labels_ok"] is True and r["config"]["global_batch"] == n


def test_two_ranks_gloo():
    pytest.importorskip("torch")  # ranks are launched with torch.distributed.run
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "10", "--warmup", "2",
           "--no-extras"]
    cp = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=str(REPO))
    assert cp.returncode == 0, cp.stderr[-3000:]
    lines = _json_lines(cp.stdout)
    assert len(lines) == 1, cp.stdout  # rank 0 only
    r = lines[0]
    assert r["n_gpus"] == 2 and r["labels_ok"] is True
    assert "2 rank(s)" in r["config"]["parallelism"]
    assert r["ms_per_step"] > 0


def test_driver_n8_command_over_fake_amdsmi(tmp_path):
    """The exact command the driver runs for the 8-GPU scaling point
    (torch.distributed.run, 8 ranks, 127.0.0.1), rehearsed on CPU: rank 0
    labels 8 MI355X GPUs through the amd-smi backend over the scriptable fake
    library (gloo for the barriers).  Checks the JSON contract and the 8-GPU
    label set: gpu.count=8 and the per-GPU xGMI links (7)."""
    import os

    pytest.importorskip("torch")  # ranks are launched with torch.distributed.run
    fake = REPO / "build" / "libfake_amdsmi.so"
    if not fake.exists():
        pytest.skip("libfake_amdsmi.so not built")
    spec = "|".join(f"bdf=0000:{0x10 + 0x10 * i:02x}:00.0;mode=SPX;parts=1;cus=256;xcds=8;vram_mib=294896;links=7"
                    for i in range(8))
    env = {**os.environ, "GFD_AMDSMI_LIBRARY": str(fake), "GFD_FAKE_AMDSMI_SPEC": spec, "GFD_BENCH_COLD_CYCLES": "2",
           "OMP_NUM_THREADS": "1"}
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "8", "--steps", "20", "--warmup", "2"]
    cp = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=str(REPO), env=env)
    assert cp.returncode == 0, cp.stderr[-3000:]
    lines = _json_lines(cp.stdout)
    assert len(lines) == 1, cp.stdout  # rank 0 only
    r = lines[0]
    assert REQUIRED <= set(r)
    assert r["n_gpus"] == 8 and r["steps"] == 20 and r["warmup"] == 2
    assert r["labels_ok"] is True, r["label_problems"]
    assert r["config"]["backend"] == "amdsmi(persistent)"
    assert "8 rank(s)" in r["config"]["parallelism"] and r["config"]["global_batch"] == 8
    assert "fake amd-smi" in r["data"]
    assert {"amdsmi.snapshot", "enumerate", "write"} <= set(r["phases_p50_ms"])
    assert r["cold_cycle"]["cycles"] == 2
    out = subprocess.run([str(REPO / "build" / "gpu-feature-discovery"), "--oneshot", "--backend=amdsmi",
                          "--output-file=", "--no-timestamp"], capture_output=True, text=True, timeout=60, env=env)
    labels = dict(ln.split("=", 1) for ln in out.stdout.splitlines())
    assert labels["amd.com/gpu.count"] == "8"
    assert labels["amd.com/gpu.xgmi.links"] == "7"
