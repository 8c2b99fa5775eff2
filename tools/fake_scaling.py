#!/usr/bin/env python3
"""Multi-GPU scaling of the amd-smi backend against the fake libamd_smi.

Each fake query busy-waits ``--latency-us`` while holding its GPU's lock
(amd-smi serialises per device), so this measures how well one labeling
cycle overlaps per-GPU queries across the worker pool for 1/2/4/8 GPUs -
the shape of the 8xMI355X case that the one-GPU boxes cannot show.

    python tools/fake_scaling.py [--latency-us 11] [--steps 300]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(REPO, "build", "libfake_amdsmi.so")
os.environ["GFD_AMDSMI_LIBRARY"] = FAKE
sys.path.insert(0, REPO)

import gpu_feature_discovery_amd as gfd  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--latency-us", type=int, default=11)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    fake = ctypes.CDLL(FAKE)
    g = gfd.native()
    g.set_quiet(True)
    root = tempfile.mkdtemp(prefix="gfd-fake-scaling-")
    for rel, text in (("opt/rocm/.info/version", "7.2.0\n"), ("proc/sys/kernel/osrelease", "6.12.12\n"),
                      ("product_name", "FAKE-NODE\n")):
        os.makedirs(os.path.dirname(os.path.join(root, rel)), exist_ok=True)
        with open(os.path.join(root, rel), "w") as f:
            f.write(text)
    os.makedirs(os.path.join(root, "sys/bus/pci/devices"), exist_ok=True)
    rows = []
    for n in (1, 2, 4, 8):
        spec = f"latency_us={a.latency_us}\n" + "".join(
            f"bdf=0000:{0x11 + 0x10 * i:02x}:00.0;mode=SPX;parts=1;cus=256;xcds=8;vram_mib=294896;links=7;virt=1\n"
            for i in range(n))
        assert fake.fake_amdsmi_configure(spec.encode()) == 0
        s = g.Session(["--backend=amdsmi", f"--sysfs-root={root}", "--output-file=", "--no-timestamp",
                       f"--machine-type-file={root}/product_name"])
        ns = s.bench(a.steps, a.warmup, False)
        ms = sorted(x / 1e6 for x in ns)
        labels = s.cycle(False)["labels"]
        assert labels["amd.com/gpu.count"] == str(n), labels
        rows.append({"gpus": n, "p50_ms": round(statistics.median(ms), 4), "p90_ms": round(ms[int(0.9 * len(ms))], 4)})
        del s
    base = rows[0]["p50_ms"]
    for r in rows:
        r["vs_1gpu"] = round(r["p50_ms"] / base, 2)
        r["serial_estimate_ms"] = round(base * r["gpus"], 4)
    print(json.dumps({"latency_us_per_call": a.latency_us, "cpus": os.cpu_count(), "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
