#!/usr/bin/env python3
"""Label-generation latency benchmark (the BASELINE.json headline metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--backend auto|amdsmi|sysfs|synthetic]

One "step" is one full labeling cycle of the daemon in its default
configuration: enumerate the node through the backend (amd-smi on a GPU
box), build every label (version, partition, xGMI, resources, SR-IOV PCI
scan) and atomically rewrite the NFD feature file.  Nothing is cached across
steps except what the daemon itself keeps between its cycles, listed with
the reason each is safe in docs/ARCHITECTURE.md ("What is kept between
cycles"): the loaded library, the persistent amd-smi session's handles and
the facts fixed until the KFD topology generation changes (ASIC identity,
virtualization mode, KFD node id and XCD count), open descriptors of sysfs
attributes, the kernel's DMI strings (copied from the firmware at boot), the
SR-IOV functions while no uevent was sent (no device added, removed, bound
or unbound), and the feature file the previous write swapped out, which the
next write rewrites whole.  Every other device value - memory, partition
modes, xGMI links, partition capabilities, versions - is read from the
driver each step.

The label set of every step is checked for correctness (count == N GPUs,
gfx950/cdna4 arch, MI355 product, HBM size, valid Kubernetes label syntax)
before timing is reported.  The in-process session runs the daemon's default
configuration: workers follow the cycle thread's L3 domain
(--cpu-affinity=follow) and block when idle; every write rewrites the file
the previous one swapped out and exchanges it with the feature file.

N>1: launched by the driver as one process per GPU under torch.distributed
(gloo, 127.0.0.1); rank 0 labels the node restricted to GPUs 0..N-1 (the
`--visible-devices` filter), every rank brackets the K steps with barriers,
and the MAX wall time over ranks is reported.  Scaling is "weak": the work
per visible GPU is fixed and total work grows with N.

Without a usable GPU (CPU container) the benchmark runs the KFD-sysfs backend
over a synthetic N-GPU MI355X tree and says so in "data"; with
GFD_AMDSMI_LIBRARY pointing at the test double (build/libfake_amdsmi.so) it
rehearses the amd-smi path on CPU.

Besides the headline (back-to-back cycles) the JSON carries the deployed
daemon's first cycle, its cycles 1 s apart on idle cores (cold_cycle), the
Job-mode process from spawn to exit, and per-phase p50s.  The timed steps
record no phases, as the daemon's without --trace-timing; the same K steps
run once more with phase tracing after the timed region, for the per-phase
p50s and their own p50 (traced_p50_ms).
"""

from __future__ import annotations

import argparse
import atexit
import gc
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gpu_feature_discovery_amd.parallel import RankGroup, env_int  # noqa: E402

METRIC = "label-file generation p50 latency (ms) + label-set correctness, 8×MI355X node"


def _percentile(xs: list[float], q: float) -> float:
    ys = sorted(xs)
    if not ys:
        return float("nan")
    k = (len(ys) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(ys) - 1)
    return ys[lo] + (ys[hi] - ys[lo]) * (k - lo)


def _check_labels(labels: dict, n_gpus: int, hardware: bool) -> list[str]:
    problems = []
    want = {
        "amd.com/gpu.count": str(n_gpus),
        "amd.com/gpu.family": "cdna4",
        "amd.com/gpu.arch": "gfx950",
        "amd.com/gpu.compute.major": "9",
        "amd.com/gpu.compute.minor": "5",
        "amd.com/gpu.replicas": "1",
    }
    for k, v in want.items():
        if labels.get(k) != v:
            problems.append(f"{k}={labels.get(k)!r} (want {v!r})")
    if "MI355" not in labels.get("amd.com/gpu.product", ""):
        problems.append(f"amd.com/gpu.product={labels.get('amd.com/gpu.product')!r}")
    mem = int(labels.get("amd.com/gpu.memory", "0") or 0)
    if not 280 * 1024 <= mem <= 300 * 1024:
        problems.append(f"amd.com/gpu.memory={mem} MiB (want ~288 GiB of HBM3E)")
    for k in ("amd.com/driver.major", "amd.com/rocm.runtime.major", "amd.com/gpu.machine", "amd.com/gfd.timestamp",
              "amd.com/gpu.partition.capable"):
        if k not in labels:
            problems.append(f"missing {k}")
    from gpu_feature_discovery_amd.utils.golden import k8s_label_problems

    problems += k8s_label_problems(labels)  # what NFD / the API server would reject
    if hardware and labels.get("amd.com/gpu.compute-units") != "256":
        problems.append(f"amd.com/gpu.compute-units={labels.get('amd.com/gpu.compute-units')!r} (want 256)")
    return problems


def _session_args(backend: str, n_gpus: int, out: str, root: str | None, extra: list[str]) -> list[str]:
    args = [f"--backend={backend}", f"--visible-devices=0-{n_gpus - 1}", f"--output-file={out}",
            "--mig-strategy=none"]
    if root:
        args.append(f"--sysfs-root={root}")
        args.append(f"--machine-type-file={root}/sys/class/dmi/id/product_name")
    return args + extra


_VARIANT = """
import json, sys
sys.path.insert(0, {repo!r})
import gpu_feature_discovery_amd as gfd
g = gfd.native(); g.set_quiet(True)
s = g.Session(json.loads(sys.argv[1]))
ns = s.bench(int(sys.argv[2]), int(sys.argv[3]), True, False)
print(json.dumps({{"ns": ns, "backend": s.backend}}))
"""


def _time_variant(args: list[str], steps: int, warmup: int) -> dict:
    """Time a daemon configuration in a fresh process (no torch, no HIP)."""
    code = _VARIANT.format(repo=os.path.dirname(os.path.abspath(__file__)))
    cp = subprocess.run([sys.executable, "-c", code, json.dumps(args), str(steps), str(warmup)], check=True,
                        capture_output=True, text=True, timeout=600)
    r = json.loads(cp.stdout.strip().splitlines()[-1])
    ms = [x / 1e6 for x in r["ns"]]
    return {"p50_ms": round(_percentile(ms, 0.5), 4), "p90_ms": round(_percentile(ms, 0.9), 4),
            "mean_ms": round(statistics.fmean(ms), 4), "backend": r["backend"]}


_ROW_PHASES = ("submit", "init", "enumerate", "label", "facts.wait", "sriov.join", "merge", "log", "write", "other",
               "facts.start", "facts(overlapped)", "write.check", "write.lease", "write.pwrite", "write.unlease",
               "write.rename", "total")


def _daemon_loop(binary: str, args: list[str], cycles: int, interval: str = "2ms",
                 env: dict | None = None) -> dict:
    """The production path: the daemon binary in loop mode, timing every
    cycle itself (--trace-timing), stopped with SIGTERM.  With a long
    `interval` every cycle after the first starts on idle, down-clocked
    cores - what a deployed DaemonSet (60 s between cycles) sees."""
    import signal

    p = subprocess.Popen([binary, f"--sleep-interval={interval}", "--trace-timing", *args], stdout=subprocess.DEVNULL,
                         stderr=subprocess.PIPE, text=True, env={**os.environ, **(env or {})})
    totals, phases, cpus, rows = [], {}, [], []
    try:
        for line in p.stderr:
            if "Timing:" in line:
                fields = dict(kv.split("=", 1) for kv in line.split("Timing:", 1)[1].split())
                cpus.append(fields.pop("cpu", ""))
                totals.append(float(fields["total"].rstrip("ms")))
                # Per cycle: the cycle thread's top-level phases and the
                # overlapped node facts (where a slow cycle spent its time).
                rows.append({k: float(v.rstrip("ms")) for k, v in fields.items()
                             if k in _ROW_PHASES or not totals[1:]})  # the first cycle: every phase
                if len(totals) > 1:
                    for k, v in fields.items():
                        phases.setdefault(k, []).append(float(v.rstrip("ms")))
                if len(totals) >= cycles:
                    break
    finally:
        p.send_signal(signal.SIGTERM)
        try:
            p.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    steady = totals[1:] or totals
    # "start,end" CPU of each cycle's thread: where the scheduler woke it.
    starts = [c.split(",")[0] for c in cpus if c]
    return {"interval": interval, "first_cycle_ms": round(totals[0], 3) if totals else None,
            "p50_ms": round(_percentile(steady, 0.5), 4), "p90_ms": round(_percentile(steady, 0.9), 4),
            "cycles": len(totals),
            # Time no phase names (total minus the top-level phases).
            "other_p50_ms": round(_percentile(phases.get("other", []), 0.5), 4),
            "cycle_cpus": cpus,
            "cpu_moves": sum(1 for a, b in zip(starts, starts[1:]) if a != b),
            "totals_ms": totals,
            "rows_ms": rows if interval != "2ms" else None,
            "first_cycle_phases_ms": rows[0] if rows else None,
            "phases_p50_ms": {k: round(_percentile(v, 0.5), 4) for k, v in phases.items() if k != "total"}}


def _cold_process(binary: str, args: list[str], runs: int) -> dict:
    """Oneshot Job mode: spawn the daemon binary per label file (the whole
    process: start, backend selection, one cycle, exit), timed from spawn to
    exit with a blocking waitpid (utils/proc.py: subprocess.run's polling
    wait quantised round 1's numbers to 3.5 / 7.5 / 31.5 / 63.5 ms)."""
    from gpu_feature_discovery_amd.utils.proc import spawn_wait_ms

    ms = [spawn_wait_ms([binary, "--oneshot", *args], timeout=60) for _ in range(runs)]
    # The first spawns after the cold-cycle measurement land on idle,
    # down-clocked cores (2-3 ms where later ones take 1.3-1.4 ms,
    # profiles/oneshot_series_r4.jsonl): the first run is reported on its own.
    return {"p50_ms": round(_percentile(ms, 0.5), 3), "p90_ms": round(_percentile(ms, 0.9), 3), "runs": runs,
            "first_ms": round(ms[0], 3), "runs_ms": [round(x, 3) for x in ms],
            "args": " ".join(a for a in args if not a.startswith(("--output-file", "--sysfs-root", "--machine")))}


def _fake_amdsmi() -> str | None:
    """GFD_AMDSMI_LIBRARY pointing at the test double: a CPU rehearsal."""
    lib = os.environ.get("GFD_AMDSMI_LIBRARY", "")
    return lib if "fake" in os.path.basename(lib) else None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=env_int("WORLD_SIZE", 1))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--backend", default="auto", help="auto | amdsmi | sysfs | synthetic")
    ap.add_argument("--no-extras", action="store_true", help="skip the secondary measurements")
    ap.add_argument("--cold-cycles", type=int, default=env_int("GFD_BENCH_COLD_CYCLES", 12),
                    help="daemon cycles 1 s apart for the cold-cycle measurement (0: skip)")
    ap.add_argument("--sysfs-root", default=None,
                    help="with --backend sysfs: read this root instead of / (tools/hybrid_root.py builds one that "
                         "shows every GPU of a shared host)")
    a = ap.parse_args()

    # Bind amd-smi to the system libdrm before anything imports PyTorch (which
    # bundles its own copy; amd-smi bound to it loses the marketing-name
    # table and pays a failed amdgpu.ids lookup on every ASIC query).  The
    # production daemon never loads PyTorch, so this is what it measures.
    import gpu_feature_discovery_amd as gfd

    gfd.native().load_amdsmi()
    dist = RankGroup()
    from gpu_feature_discovery_amd.ops import Labeler
    from gpu_feature_discovery_amd.utils import synth

    g = gfd.native()
    g.set_quiet(True)
    n = a.gpus

    tmp = tempfile.mkdtemp(prefix="gfd-bench-")
    atexit.register(shutil.rmtree, tmp, True)
    out = os.path.join(tmp, "features.d", "gfd")
    os.makedirs(os.path.dirname(out), exist_ok=True)

    # Decide the backend on rank 0 (only rank 0 talks to the driver).
    hardware = False
    root = None
    backend = a.backend
    if dist.rank == 0:
        if backend in ("auto", "amdsmi"):
            try:
                devs = Labeler(["--backend=amdsmi", f"--visible-devices=0-{n - 1}"]).devices()
                hardware = len(devs) >= n
                if not hardware and a.backend == "amdsmi":
                    raise SystemExit(f"amd-smi sees {len(devs)} GPU(s), fewer than --gpus {n}")
            except g.GfdError:
                if a.backend == "amdsmi":
                    raise
                hardware = False
            backend = "amdsmi" if hardware else "synthetic"
        if backend in ("synthetic",):
            root = os.path.join(tmp, "root")
            synth.make_mi355x_node(root, n_gpus=n, seed=1234)
        elif backend == "sysfs":
            hardware = True
            root = a.sysfs_root
    backend = dist.broadcast_obj(backend)
    hardware = dist.broadcast_obj(hardware)

    session = None
    labels_ok, problems, labels = True, [], {}
    if dist.rank == 0:
        sess_backend = "sysfs" if backend == "synthetic" else backend
        args = _session_args(sess_backend, n, out, root, [])
        session = Labeler(args)
        labels = session.cycle(write=True).labels
        problems = _check_labels(labels, n, hardware)
        labels_ok = not problems
        # Warmup (untimed), in native code.  The cycles record no phases, as
        # the daemon's without --trace-timing (phase tracing reads the clock
        # twice per phase, ~1.5 us of a cycle): the phases come from K traced
        # steps after the timed region.
        session.bench(0, a.warmup, True, False)

    # Timed region: exactly K steps, bracketed by barrier + synchronize.
    dist.sync()
    t0 = time.perf_counter_ns()
    ms: list[float] = []
    if dist.rank == 0:
        ms = session.bench(a.steps, 0, True, False)
    dist.sync()
    wall_ms = (time.perf_counter_ns() - t0) / 1e6
    wall_ms = dist.max(wall_ms)

    if dist.rank == 0:
        p50 = _percentile(ms, 0.5)
        backend_name = session.backend
        # The same K steps again, traced: where a cycle spends its time (and
        # what tracing costs, traced_p50_ms - value).
        traced_ms = session.bench(a.steps, 0, True, True)
        bench_phases = session.bench_phases()
        phases = {name: round(_percentile(v, 0.5), 4) for name, v in bench_phases.items()}
        # In how many of the K timed steps each phase occurred (a step that
        # created its own temporary file, took over the SR-IOV lookup...).
        phases_n = {name: len(v) for name, v in bench_phases.items() if len(v) != a.steps}
        # Release the persistent amd-smi session before measuring variants
        # that must pay amdsmi_init themselves.
        del session
        gc.collect()
        extras: dict = {}
        cold, first_cycle = None, None
        fake = _fake_amdsmi()
        if not a.no_extras:
            # The daemon as the DaemonSet runs it: --backend=auto (amd-smi,
            # initialised in the background while KFD labels the first cycle).
            loop_args = _session_args("auto", n, out, root, [])
            try:
                binary = str(gfd.binary_path())
                runs = max(15, min(30, a.steps // 10))
                extras["daemon_loop"] = _daemon_loop(binary, loop_args, max(20, min(a.steps, 300)))
                first_cycle = extras["daemon_loop"]["first_cycle_ms"]
                # Deployed cadence: cycles after >= 1 s of idle (the daemon
                # sleeps 60 s), each starting on cold, down-clocked cores.
                if a.cold_cycles > 1:
                    cold = _daemon_loop(binary, loop_args, a.cold_cycles, interval="1s")
                if backend == "amdsmi":
                    extras["amdsmi_per_cycle_session"] = _time_variant(
                        _session_args("amdsmi", n, out, None, ["--amdsmi-session=per-cycle"]), max(10, a.steps // 10), 2)
                    extras["sysfs_backend"] = _time_variant(_session_args("sysfs", n, out, None, []), a.steps, a.warmup)
                # Job mode as deployed (the Job template: --backend=auto),
                # the whole process from spawn to exit.
                extras["oneshot_process"] = _cold_process(binary, _session_args("auto", n, out, root, []), runs)
                if backend == "amdsmi":
                    extras["oneshot_process_amdsmi"] = _cold_process(binary, _session_args("amdsmi", n, out, None, []),
                                                                     runs)
            except (FileNotFoundError, subprocess.SubprocessError, ValueError) as e:
                extras["error"] = str(e)
        if backend == "amdsmi" and fake:
            data = f"CPU rehearsal: fake amd-smi library ({os.path.basename(fake)}), {n} scripted MI355X GPU(s)"
        elif backend == "amdsmi":
            data = ("real MI355X, amd-smi backend: processor handles, KFD ids, identity, partition modes, memory, "
                    "xGMI links and capabilities kept for the persistent amd-smi session, which every step checks "
                    "against the KFD topology generation (a partition/NPS switch or driver reload re-initialises "
                    "it); driver and ROCm versions, the SR-IOV state (uevent counter) and the feature file read or "
                    "written every step")
        elif backend == "sysfs":
            data = f"real MI355X via KFD sysfs under {root}" if root else "real MI355X via KFD sysfs"
        else:
            data = f"synthetic {n}-GPU MI355X sysfs tree (random device IDs), no GPU available"
        result = {
            "metric": METRIC,
            "value": round(p50, 4),
            "unit": "ms",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(wall_ms / max(a.steps, 1), 4),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "n/a",
            "data": data,
            "config": {
                "model": f"{n}xMI355X SPX/NPS1 node, amd.com label set",
                "global_batch": n,
                "seq_len": None,
                "parallelism": f"1 labeler for {n} visible GPU(s); {dist.world} rank(s)",
                "backend": backend_name,
                "strategy": "none",
            },
            "p90_ms": round(_percentile(ms, 0.9), 4),
            "p99_ms": round(_percentile(ms, 0.99), 4),
            "max_ms": round(max(ms), 4) if ms else None,
            "mean_ms": round(statistics.fmean(ms), 4) if ms else None,
            # The K steps once more with phase tracing (after the timed
            # region): their p50, and the per-phase p50s - what an N-GPU
            # cycle spends where (the scaling curve's explanation).
            "traced_p50_ms": round(_percentile(traced_ms, 0.5), 4),
            "phases_p50_ms": phases,
            "phases_n": phases_n,
            # The deployed daemon's first cycle (library init included) and
            # its cycles after an idle second (see _daemon_loop).
            "first_cycle_ms": first_cycle,
            "cold_cycle": cold,
            "oneshot_process_p50_ms": extras.get("oneshot_process", {}).get("p50_ms"),
            "labels_ok": labels_ok,
            "label_problems": problems,
            "n_labels": len(labels),
            "extras": extras,
        }
        print(json.dumps(result))
    dist.close()
    return 0 if labels_ok else 1


if __name__ == "__main__":
    sys.exit(main())
