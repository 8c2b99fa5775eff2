"""bench.py contract tests on CPU (synthetic MI355X sysfs tree).

The driver runs ``python bench.py --gpus N --steps K --warmup W`` (N>1 under
torch.distributed.run, one rank per GPU); rank 0 must print exactly one JSON
line with the contract's fields.  The multi-rank path is exercised with the
gloo backend and world_size 2 on 127.0.0.1.
"""

from __future__ import annotations

import json
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
    cp = subprocess.run([sys.executable, "bench.py", "--steps", "30", "--warmup", "3", "--backend", "synthetic"],
                        capture_output=True, text=True, timeout=300, cwd=str(REPO))
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
    assert {"init", "enumerate", "label", "write"} <= set(r["extras"]["phases_ms"])
    assert r["extras"]["oneshot_process"]["p50_ms"] > 0


@pytest.mark.parametrize("n", [2, 4, 8])
def test_synthetic_scaling_labels(n):
    cp = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "10", "--warmup", "1", "--backend",
                         "synthetic", "--no-extras"], capture_output=True, text=True, timeout=300, cwd=str(REPO))
    assert cp.returncode == 0, cp.stderr[-3000:]
    r = _json_lines(cp.stdout)[0]
    assert r["n_gpus"] == n and r["labels_ok"] is True and r["config"]["global_batch"] == n


def test_two_ranks_gloo():
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
