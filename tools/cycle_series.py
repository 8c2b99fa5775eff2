#!/usr/bin/env python3
"""Per-cycle view of the headline bench: which cycles are slow, and whether
their write found a prepared temporary file.

    python tools/cycle_series.py [--steps 200] [--warmup 20] [--backend amdsmi] [--runs 3]

Runs the same in-process Session.bench as bench.py (amd-smi backend on a GPU
box, KFD sysfs otherwise) and prints, per run: p50/p90/mean, how many cycles
took more than 1.5x the p50 and where they fall (first/second half), and
how many writes took a prepared file (write.take) vs created one
(write.create).
"""

from __future__ import annotations

import argparse
import os
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import gpu_feature_discovery_amd as gfd  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--backend", default="amdsmi")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--sysfs-root", default=None, help="with --backend sysfs: a synthetic tree (CPU check)")
    a = ap.parse_args()
    g = gfd.native()
    g.load_amdsmi()
    g.set_quiet(True)
    for run in range(a.runs):
        d = tempfile.mkdtemp(prefix="gfd-series-")
        out = os.path.join(d, "features.d", "gfd")
        os.makedirs(os.path.dirname(out))
        args = [f"--backend={a.backend}", "--visible-devices=0-0", f"--output-file={out}", "--mig-strategy=none"]
        if a.sysfs_root:
            args += [f"--sysfs-root={a.sysfs_root}", f"--machine-type-file={a.sysfs_root}/sys/class/dmi/id/product_name"]
        s = g.Session(args)
        ns = s.bench(a.steps, a.warmup, True)
        ph = s.bench_phases()
        del s
        ms = [x / 1e6 for x in ns]
        p50 = statistics.median(ms)
        slow = [i for i, x in enumerate(ms) if x > 1.5 * p50]
        half = len(ms) // 2
        print(f"run {run}: p50 {p50:.4f} p90 {sorted(ms)[int(0.9 * (len(ms) - 1))]:.4f} mean {statistics.fmean(ms):.4f} ms; "
              f"{len(slow)} cycles > 1.5x p50 ({sum(i < half for i in slow)} in the first half, first at {slow[:8]}); "
              f"writes: {len(ph.get('write.take', []))} took a prepared file, {len(ph.get('write.create', []))} created one "
              f"(create p50 {statistics.median(ph['write.create']) / 1e3 if ph.get('write.create') else 0:.1f} us)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
