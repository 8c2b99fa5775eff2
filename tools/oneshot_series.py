#!/usr/bin/env python3
"""Job-mode process wall times in launch order, for a few argument sets.

    python tools/oneshot_series.py [--runs 30]

bench.py's `oneshot_process` takes the p50 of a handful of runs of the Job's
command; this prints every run of that command and of variants of it, so a
warm-up trend (page cache, first exec of the binary) or an argument that
costs time shows up.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gpu_feature_discovery_amd.utils.proc import spawn_wait_ms  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=30)
    a = ap.parse_args()
    binary = os.path.join(REPO, "build", "gpu-feature-discovery")
    tmp = tempfile.mkdtemp(prefix="gfd-series-")
    out = os.path.join(tmp, "features.d", "gfd")
    os.makedirs(os.path.dirname(out))
    variants = {
        "bench": ["--backend=auto", "--visible-devices=0-0", f"--output-file={out}", "--mig-strategy=none"],
        "no-filter": ["--backend=auto", f"--output-file={out}", "--mig-strategy=none"],
        "repo-dir": ["--backend=auto", "--visible-devices=0-0", f"--output-file={REPO}/gpurun_out/series_gfd"],
        "true": None,
    }
    for name, args in variants.items():
        argv = ["/bin/true"] if args is None else [binary, "--oneshot", *args]
        xs = [round(spawn_wait_ms(argv, timeout=60), 3) for _ in range(a.runs)]
        print(json.dumps({"variant": name, "p50_ms": round(statistics.median(xs), 3),
                          "p50_first5_ms": round(statistics.median(xs[:5]), 3), "runs": xs}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
