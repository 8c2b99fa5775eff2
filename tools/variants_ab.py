#!/usr/bin/env python3
"""Same-box, alternated A/B of daemon variants in the three regimes the
driver records: the headline (bench.py --steps 20 --warmup 5, a fresh
process per run), cycles 1 s apart (the daemon binary, tools/cold_cycle.py)
and the oneshot Job process (spawn to exit).

    python tools/variants_ab.py --variant NAME=ENV=V,ENV=V ... [--reps 4]
                                [--modes headline,cold,job] [--cold-cycles 8]

A variant is a set of environment settings (experiment switches, or
BIN=<path> / TREE=<dir> for a staged older build).  Runs alternate
variant by variant within each repetition, so a drift of the box hits all
of them alike.  One JSON line per run, then a summary per variant and mode.
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import statistics
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gpu_feature_discovery_amd.utils.proc import spawn_wait_ms  # noqa: E402

PHASES = ("submit", "init", "enumerate", "label", "facts", "facts.wait", "sriov.self", "sriov", "sriov.join", "merge",
          "write", "write.create", "write.reuse", "write.data", "write.rename", "facts(overlapped)",
          "facts.start", "facts.machine", "facts.driver", "facts.runtime", "pci.bound(kept)", "other")


def parse_variant(text: str) -> tuple[str, dict]:
    name, _, rest = text.partition("=")
    env = {}
    for kv in filter(None, rest.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    return name, env


def headline(env: dict, steps: int, warmup: int) -> dict:
    tree = env.get("TREE", REPO)
    e = {**os.environ, **{k: v for k, v in env.items() if k not in ("TREE", "BIN")}}
    cp = subprocess.run([sys.executable, "bench.py", "--steps", str(steps), "--warmup", str(warmup), "--no-extras",
                         "--cold-cycles", "0"], cwd=tree, env=e, capture_output=True, text=True, timeout=300)
    if cp.returncode != 0:
        raise RuntimeError(cp.stderr[-2000:])
    d = json.loads(cp.stdout.strip().splitlines()[-1])
    p = d["phases_p50_ms"]
    return {"value": d["value"], "p90": d["p90_ms"], "n": d.get("phases_n", {}), **{k: p[k] for k in PHASES if k in p}}


def cold(env: dict, cycles: int, interval: str) -> dict:
    binary = env.get("BIN", os.path.join(env.get("TREE", REPO), "build", "gpu-feature-discovery"))
    e = {**os.environ, **{k: v for k, v in env.items() if k not in ("TREE", "BIN")}}
    out = os.path.join(tempfile.mkdtemp(prefix="gfd-ab-"), "features.d", "gfd")
    p = subprocess.Popen([binary, f"--sleep-interval={interval}", "--trace-timing", f"--output-file={out}",
                          "--backend=auto", "--visible-devices=0-0", "--mig-strategy=none"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=e)
    rows = []
    try:
        for line in p.stderr:
            if "Timing:" not in line:
                continue
            f = dict(kv.split("=", 1) for kv in line.split("Timing:", 1)[1].split())
            f.pop("cpu", None)
            rows.append({k: float(v.rstrip("ms")) for k, v in f.items()})
            if len(rows) >= cycles:
                break
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=30)
    steady = rows[1:]
    med = {k: round(statistics.median([r.get(k, 0.0) for r in steady]), 4) for k in PHASES + ("total",)
           if any(k in r for r in steady)}
    return {"value": med.get("total"), "first": rows[0]["total"] if rows else None, "totals": [r["total"] for r in rows],
            **{k: v for k, v in med.items() if k != "total"}}


def job(env: dict, runs: int) -> dict:
    binary = env.get("BIN", os.path.join(env.get("TREE", REPO), "build", "gpu-feature-discovery"))
    e = {**os.environ, **{k: v for k, v in env.items() if k not in ("TREE", "BIN")}}
    out = os.path.join(tempfile.mkdtemp(prefix="gfd-ab-"), "features.d", "gfd")
    os.makedirs(os.path.dirname(out))
    argv = [binary, "--oneshot", "--backend=auto", "--visible-devices=0-0", f"--output-file={out}",
            "--mig-strategy=none"]
    xs = [round(spawn_wait_ms(argv, timeout=60, env=e), 3) for _ in range(runs)]
    return {"value": round(statistics.median(xs), 3), "runs": xs}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--modes", default="headline,cold,job")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cold-cycles", type=int, default=8)
    ap.add_argument("--interval", default="1s")
    ap.add_argument("--job-runs", type=int, default=10)
    a = ap.parse_args()
    variants = [parse_variant(v) for v in a.variant]
    modes = a.modes.split(",")
    results: dict = {}
    for rep in range(a.reps):
        for mode in modes:
            for name, env in variants:
                if mode == "headline":
                    r = headline(env, a.steps, a.warmup)
                elif mode == "cold":
                    r = cold(env, a.cold_cycles, a.interval)
                else:
                    r = job(env, a.job_runs)
                results.setdefault((mode, name), []).append(r)
                print(json.dumps({"mode": mode, "variant": name, "rep": rep, **r}), flush=True)
    for (mode, name), rs in results.items():
        vals = [r["value"] for r in rs if r["value"] is not None]
        keys = sorted({k for r in rs for k in r if k in PHASES})
        print(json.dumps({"summary": mode, "variant": name, "median": round(statistics.median(vals), 4) if vals else None,
                          "values": vals,
                          "phases": {k: round(statistics.median([r.get(k, 0.0) for r in rs]), 4) for k in keys}}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
