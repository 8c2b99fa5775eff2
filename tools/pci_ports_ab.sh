#!/bin/bash
# A/B of skipping AMD functions bound to pcieport in the cold PCI scan: Job
# processes (--oneshot, null and auto backends) with GFD_PCI_PORTS=read vs
# the default, alternated, spawn to exit with a blocking waitpid.
# Usage (GPU box): tools/pci_ports_ab.sh [outdir-name] [reps]
set -o pipefail
out=gpurun_out/${1:-pci_ports_ab}
mkdir -p "$out"
python3 - "$out" "${2:-3}" <<'PY' | tee "$out/ab.txt"
import os, statistics, sys
sys.path.insert(0, ".")
from gpu_feature_discovery_amd.utils.proc import spawn_wait_ms
out, reps = sys.argv[1], int(sys.argv[2])
binary = "./build/gpu-feature-discovery"
amd = [l.split("\t") for l in open("/proc/bus/pci/devices") if l.split("\t")[1].startswith("1002")]
print(f"# {sum(1 for _ in open('/proc/bus/pci/devices'))} PCI functions, {len(amd)} AMD, "
      f"{sum(1 for f in amd if f[-1].strip() == 'pcieport')} of them bound to pcieport")
for r in range(reps):
    for mode in ("read", "skip"):
        env = dict(os.environ)
        env.pop("GFD_PCI_PORTS", None)
        if mode == "read":
            env["GFD_PCI_PORTS"] = "read"
        for backend in ("null", "auto"):
            xs = sorted(spawn_wait_ms([binary, "--oneshot", f"--backend={backend}", f"--output-file={out}/gfd"], timeout=60, env=env)
                        for _ in range(30))
            print(f"rep {r} ports={mode:4s} oneshot {backend:4s}: p50 {statistics.median(xs):.3f} ms  p90 {xs[27]:.3f} ms")
PY
