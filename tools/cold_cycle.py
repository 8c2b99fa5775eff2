#!/usr/bin/env python3
"""Cycle latency of the daemon as deployed: a real sleep between cycles
(cores idle, workers parked, caches cold), read from its own --trace-timing.

    python tools/cold_cycle.py [--interval 1s] [--cycles 9] [--backend auto]
                               [--variants follow,none,l3] [--reps 3] [--rows]

Each variant is a daemon flag set (`--cpu-affinity=<v>` for a bare name, or
a literal list of flags and NAME=value environment settings, space-separated,
e.g. "GFD_CYCLE_TASKS=inline"); variants are run alternately, `reps`
times each, so a box-wide drift hits all of them alike.  Prints one JSON
line per run and a summary per variant: p50 of the cycle total, of the
unattributed time (`other`) and of every phase, over the cycles after the
first, plus how often the cycle thread woke on another CPU.
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

ROWS = False  # --rows: every cycle's full Timing fields in the per-run line
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_once(binary: str, flags: list[str], interval: str, cycles: int, extra: list[str]) -> dict:
    out = os.path.join(tempfile.mkdtemp(prefix="gfd-cold-"), "gfd")
    # NAME=value tokens of a variant are environment variables; BIN=<path>
    # runs another daemon binary (e.g. an older build staged for an A/B).
    env = dict(os.environ)
    for f in [f for f in flags if not f.startswith("-") and "=" in f]:
        k, v = f.split("=", 1)
        if k == "BIN":
            binary = v
        else:
            env[k] = v
    flags = [f for f in flags if f.startswith("-")]
    p = subprocess.Popen([binary, f"--sleep-interval={interval}", "--trace-timing", f"--output-file={out}", *extra,
                          *flags], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=env)
    rows = []
    try:
        for line in p.stderr:
            if "Timing:" not in line:
                continue
            fields = dict(kv.split("=", 1) for kv in line.split("Timing:", 1)[1].split())
            cpu = fields.pop("cpu", "")
            row = {k: float(v.rstrip("ms")) for k, v in fields.items()}
            row["cpu"] = cpu
            rows.append(row)
            if len(rows) >= cycles:
                break
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=30)
    steady = rows[1:]
    starts = [r["cpu"].split(",")[0] for r in rows]
    phases = {}
    for r in steady:
        for k, v in r.items():
            if k != "cpu":
                phases.setdefault(k, []).append(v)
    return {"first_ms": rows[0]["total"] if rows else None,
            "p50_ms": round(statistics.median(phases["total"]), 4) if steady else None,
            "other_p50_ms": round(statistics.median(phases.get("other", [0])), 4) if steady else None,
            "cpu_moves": sum(1 for a, b in zip(starts, starts[1:]) if a != b),
            "cpus": [r["cpu"] for r in rows],
            "totals": [r["total"] for r in rows],
            "rows": rows if ROWS else None,
            "phases_p50_ms": {k: round(statistics.median(v), 4) for k, v in phases.items()}}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--interval", default="1s")
    ap.add_argument("--cycles", type=int, default=9)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--sysfs-root", default=None)
    ap.add_argument("--visible-devices", default="")
    ap.add_argument("--variants", default="follow", help="comma-separated --cpu-affinity values or flag lists")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--rows", action="store_true", help="print every cycle's phases")
    ap.add_argument("--binary", default=os.path.join(REPO, "build", "gpu-feature-discovery"))
    a = ap.parse_args()
    global ROWS
    ROWS = a.rows
    extra = [f"--backend={a.backend}"]
    if a.visible_devices:
        extra.append(f"--visible-devices={a.visible_devices}")
    if a.sysfs_root:
        extra += [f"--sysfs-root={a.sysfs_root}", f"--machine-type-file={a.sysfs_root}/sys/class/dmi/id/product_name"]
    variants = [v.strip() for v in a.variants.split(",") if v.strip()]
    per: dict[str, list[dict]] = {v: [] for v in variants}
    for rep in range(a.reps):
        for v in variants:
            flags = v.split() if " " in v or v.startswith("--") or "=" in v else [f"--cpu-affinity={v}"]
            r = run_once(a.binary, flags, a.interval, a.cycles, extra)
            per[v].append(r)
            print(json.dumps({"variant": v, "rep": rep, **r}), flush=True)
    for v, runs in per.items():
        tot = [t for r in runs for t in r["totals"][1:]]
        oth = [r["other_p50_ms"] for r in runs]
        print(json.dumps({"summary": v, "runs": len(runs), "cycles": len(tot),
                          "p50_ms": round(statistics.median(tot), 4) if tot else None,
                          "run_p50s_ms": [r["p50_ms"] for r in runs], "other_p50s_ms": oth,
                          "cpu_moves": [r["cpu_moves"] for r in runs]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
