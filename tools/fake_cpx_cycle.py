#!/usr/bin/env python3
"""Cycle cost of the amd-smi backend on CPX nodes (BASELINE config 4), which
the one-GPU pool boxes cannot be switched into: a synthetic N-GPU CPX tree
(8 KFD partition nodes per GPU) and the fake libamd_smi configured to match
it, every non-trivial fake call busy-waiting ``--latency-us`` under its GPU's
lock (amd-smi serialises per device; ~10-20 us per call measured on MI355X,
profiles/amdsmi_api_latency_probe.txt).

Compares the library path (GFD_AMDSMI_SYSFS=0: memory, partition modes and
KFD info through amd-smi for every partition, every cycle) with the default
path (partition modes from the parent's amdgpu attributes, per-partition
facts cached per session).  CPU measurement; says nothing about absolute
MI355X latencies beyond the modelled call cost.

    python tools/fake_cpx_cycle.py [--latency-us 15] [--steps 200]
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gpu_feature_discovery_amd.utils import synth  # noqa: E402

_RUN = """
import json, statistics, sys
sys.path.insert(0, {repo!r})
import gpu_feature_discovery_amd as gfd
g = gfd.native(); g.set_quiet(True)
s = g.Session(json.loads(sys.argv[1]))
ns = sorted(s.bench(int(sys.argv[2]), 20, False))
labels = s.cycle(False)["labels"]
print(json.dumps({{"p50_ms": round(ns[len(ns) // 2] / 1e6, 4), "p90_ms": round(ns[int(0.9 * len(ns))] / 1e6, 4),
                  "count": labels.get("amd.com/partition-cpx.1xcd.36gb.count")}}))
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--latency-us", type=int, default=15)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    fake = os.path.join(REPO, "build", "libfake_amdsmi.so")
    rows = []
    for n in (1, 2, 4, 8):
        spec = synth.NodeSpec(gpus=[synth.GpuSpec(compute_partition="CPX") for _ in range(n)], seed=40 + n)
        root = synth.make_node(tempfile.mkdtemp(prefix="gfd-cpx-"), spec)
        args = ["--backend=amdsmi", f"--sysfs-root={root}", "--output-file=", "--no-timestamp",
                "--mig-strategy=mixed", f"--machine-type-file={root}/sys/class/dmi/id/product_name"]
        row = {"gpus": n, "partitions": 8 * n}
        for name, extra in (("library_path", {"GFD_AMDSMI_SYSFS": "0"}), ("default", {})):
            env = {**os.environ, "GFD_AMDSMI_LIBRARY": fake,
                   "GFD_FAKE_AMDSMI_SPEC": synth.fake_amdsmi_spec(root, spec, a.latency_us).replace("\n", "|"),
                   **extra}
            cp = subprocess.run([sys.executable, "-c", _RUN.format(repo=REPO), json.dumps(args), str(a.steps)],
                                env=env, capture_output=True, text=True, timeout=600, check=True)
            r = json.loads(cp.stdout.strip().splitlines()[-1])
            assert r["count"] == str(8 * n), r
            row[name] = {"p50_ms": r["p50_ms"], "p90_ms": r["p90_ms"]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
