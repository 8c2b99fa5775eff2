#!/bin/bash
# A/B of the cold SR-IOV PCI scan in a oneshot process: procfs vendor table
# (default) vs per-function sysfs vendor reads over the worker pool
# (GFD_PCI_COLD=sysfs).  Whole-process wall time and the in-process trace.
set -o pipefail
out=gpurun_out/${1:-pci_cold_ab}
mkdir -p "$out"
python3 - "$out" <<'PY' > "$out/ab.txt" 2>&1
import os, statistics, subprocess, sys, time
out = sys.argv[1]
b = "./build/gpu-feature-discovery"
for mode in ("proc", "sysfs", "proc", "sysfs"):
    env = dict(os.environ, GFD_PCI_COLD=mode)
    ws, traces = [], []
    for i in range(30):
        t0 = time.perf_counter_ns()
        cp = subprocess.run([b, "--oneshot", "--backend=null", "--trace-timing", f"--output-file={out}/gfd"], env=env,
                            capture_output=True, text=True, check=True)  # no timeout: it would poll (utils/proc.py)
        ws.append((time.perf_counter_ns() - t0) / 1e6)
        traces.append(next(l for l in cp.stderr.splitlines() if "Timing:" in l))
    print(f"{mode:6s} process p50 {statistics.median(ws):.3f} ms; a cycle: {traces[len(traces)//2].split('Timing: ')[1]}")
PY
rc=$?
cat "$out/ab.txt"
exit $rc
