#!/usr/bin/env python3
"""In-process write sub-phases on the file system of DIR: python tools/write_ext4_session.py DIR CYCLES
(with GFD_WRITE_PREALLOC / GFD_WRITE_PREPARE set per run; profiles/write_ext4_ab.txt)."""
import sys, os, statistics
sys.path.insert(0, "/root/repo")
import gpu_feature_discovery_amd as gfd
from gpu_feature_discovery_amd.utils import synth
g = gfd.native(); g.set_quiet(True)
base = sys.argv[1]
root = base + "/root"
synth.make_mi355x_node(root, n_gpus=1, seed=1)
out = base + "/features.d/gfd"
os.makedirs(os.path.dirname(out), exist_ok=True)
s = g.Session(["--backend=sysfs", f"--sysfs-root={root}", f"--output-file={out}", f"--machine-type-file={root}/sys/class/dmi/id/product_name"])
ns = s.bench(int(sys.argv[2]), 5, True)
ph = s.bench_phases()
print(os.environ.get("GFD_WRITE_PREALLOC", "default"), os.environ.get("GFD_WRITE_PREPARE", "default"), "cycle p50 %.4f ms max %.3f ms" % (statistics.median(ns)/1e6, max(ns)/1e6), end=" |")
for k in sorted(ph):
    if k.startswith("write."):
        v = ph[k]; print(" %s p50 %.1f us" % (k, statistics.median(v)/1e3), end="")
print()
