#!/usr/bin/env python3
"""Same-box, alternated A/B of oneshot Jobs, phase by phase: spawns
`--oneshot --backend=auto --trace-timing` under each variant's environment
(NAME=ENV=V,ENV=V; a build with experiment switches read from the
environment), round-robin, and reports the p50 of the Job's `pci.bound`,
`sriov` and `total` phases and of the process wall time.  Made for the SR-IOV
scan's per-function reads, which a Job runs cold on its one thread
(profiles/sriov_scan_ab_r5.txt).

    python tools/sriov_scan_ab.py --variant base= --variant x=GFD_EXP_SWITCH=on --runs 60
"""

from __future__ import annotations

import argparse
import json
import os
import re
import statistics
import subprocess
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
BIN = REPO / "build" / "gpu-feature-discovery"


def one(env: dict, out: str) -> dict:
    t0 = time.perf_counter()
    p = subprocess.run([str(BIN), "--oneshot", "--backend=auto", "--trace-timing", f"--output-file={out}"],
                       env={**os.environ, **env}, capture_output=True, text=True, timeout=60)
    wall = (time.perf_counter() - t0) * 1e3
    if p.returncode != 0:
        raise SystemExit(f"job failed: {p.stderr[-500:]}")
    line = next(x for x in p.stderr.splitlines() if "Timing:" in x)
    ph = {k: float(v) for k, v in re.findall(r"([\w.()]+)=([0-9.]+)ms", line)}
    return {"wall": wall, **ph}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--runs", type=int, default=40)
    a = ap.parse_args()
    variants = []
    for v in a.variant:
        name, _, spec = v.partition("=")
        env = dict(kv.split("=", 1) for kv in spec.split(",") if kv) if spec else {}
        variants.append((name, env))
    out = os.path.join(tempfile.mkdtemp(prefix="gfd-sriov-ab-"), "gfd")
    rows: dict[str, list[dict]] = {n: [] for n, _ in variants}
    for i in range(a.runs):
        for name, env in (variants if i % 2 == 0 else variants[::-1]):
            rows[name].append(one(env, out))
        if i % 10 == 9:
            print(json.dumps({"progress": i + 1}), flush=True)
    for name, _ in variants:
        r = rows[name]
        med = {k: round(statistics.median(x[k] for x in r if k in x), 4) for k in ("pci.bound", "sriov", "total", "wall")}
        q = {k + "_p25_p75": [round(statistics.quantiles([x[k] for x in r], n=4)[0], 4),
                              round(statistics.quantiles([x[k] for x in r], n=4)[2], 4)] for k in ("pci.bound", "total")}
        print(json.dumps({"summary": name, "runs": len(r), **med, **q}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
