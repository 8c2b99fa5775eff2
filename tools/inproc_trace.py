#!/usr/bin/env python3
"""Per-call amd-smi timing of in-process labeling cycles, with and without
PyTorch in the process (and in which load order), and of the KFD-sysfs
backend ("sysfs" column).

    python tools/inproc_trace.py [cycles]
"""

from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, json, statistics
sys.path.insert(0, {repo!r})
mode = sys.argv[1]; n = int(sys.argv[2])
import gpu_feature_discovery_amd as gfd
g = gfd.native(); g.set_quiet(True)
if mode == "torch-first":
    import torch; torch.cuda.device_count()
if mode == "amdsmi-first":
    g.load_amdsmi(); import torch; torch.cuda.device_count()
backend = "sysfs" if mode == "sysfs" else "amdsmi"
s = g.Session(["--backend=" + backend, "--output-file=/tmp/gfd-inproc/gfd"])
acc = {{}}
for i in range(n):
    r = s.cycle(True)
    if i < 10: continue
    for k, v in r["phases"]:
        acc.setdefault(k, []).append(v / 1e3)
    acc.setdefault("total", []).append(r["total_ns"] / 1e3)
print(json.dumps({{k: round(statistics.median(v), 1) for k, v in acc.items()}}))
"""


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    os.makedirs("/tmp/gfd-inproc", exist_ok=True)
    env = {**os.environ, "GFD_AMDSMI_CALL_TRACE": "1"}
    rows = {}
    for mode in ("no-torch", "amdsmi-first", "torch-first", "sysfs"):
        cp = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO), mode, str(n)], capture_output=True,
                            text=True, timeout=600, env=env)
        if cp.returncode != 0:
            rows[mode] = {"error": cp.stderr[-500:]}
            continue
        rows[mode] = json.loads(cp.stdout.strip().splitlines()[-1])
    keys = sorted({k for r in rows.values() for k in r if k != "error"})
    print(f"{'us (median)':45s}" + "".join(f"{m:>14s}" for m in rows))
    for k in keys:
        print(f"{k:45s}" + "".join(f"{rows[m].get(k, float('nan')):>14}" for m in rows))


if __name__ == "__main__":
    main()
