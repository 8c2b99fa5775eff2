#!/usr/bin/env python3
"""Where a cold Job process spends its time: the Job's command run N times,
each after an idle pause (as a Job lands on an idle node), with the
daemon's own --trace-timing phases and process timeline next to the spawn-
to-exit wall time.

    python tools/job_cold.py [--runs 10] [--pause 1.0] [extra daemon flags...]
"""

from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--pause", type=float, default=1.0)
    a, extra = ap.parse_known_args()
    binary = os.path.join(REPO, "build", "gpu-feature-discovery")
    out = os.path.join(tempfile.mkdtemp(prefix="gfd-job-"), "features.d", "gfd")
    os.makedirs(os.path.dirname(out))
    argv = [binary, "--oneshot", "--trace-timing", "--backend=auto", "--visible-devices=0-0", f"--output-file={out}",
            "--mig-strategy=none", *extra]
    rows = []
    for _ in range(a.runs):
        time.sleep(a.pause)
        t0 = time.perf_counter_ns()
        cp = subprocess.run(argv, capture_output=True, text=True)
        wall = (time.perf_counter_ns() - t0) / 1e6
        row = {"wall_ms": round(wall, 3)}
        for line in cp.stderr.splitlines():
            if "Process timing:" in line:
                for kv in line.split("Process timing:", 1)[1].split():
                    k, v = kv.split("=", 1)
                    if k != "main_at":
                        row["proc." + k] = float(v.rstrip("ms"))
            elif "Timing:" in line:
                for kv in line.split("Timing:", 1)[1].split():
                    k, v = kv.split("=", 1)
                    if k != "cpu":
                        row[k] = float(v.rstrip("ms"))
        rows.append(row)
        print(json.dumps(row), flush=True)
    keys = sorted({k for r in rows for k in r})
    print(json.dumps({"p50": {k: round(statistics.median([r[k] for r in rows if k in r]), 4) for k in keys}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
