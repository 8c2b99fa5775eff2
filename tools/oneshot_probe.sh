#!/bin/bash
# Where a cold oneshot cycle's time goes (Job mode): process start, and the
# daemon's own per-phase trace for both backends; PCI domain layout.
set -o pipefail
out=gpurun_out/${1:-oneshot}
mkdir -p $out
{
  echo "## PCI functions per domain"; ls /sys/bus/pci/devices | cut -d: -f1 | sort | uniq -c
  echo "## /proc/bus/pci/devices lines"; wc -l < /proc/bus/pci/devices
  echo "## AMD (0x1002) functions"; grep -l 0x1002 /sys/bus/pci/devices/*/vendor | wc -l
  python3 - <<'PY'
import subprocess, time, statistics
def t(cmd, n=30):
    xs = []
    for _ in range(n):
        a = time.perf_counter(); subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True); xs.append((time.perf_counter() - a) * 1e3)
    return round(statistics.median(xs), 3)
print("## exec p50 ms: /bin/true", t(["/bin/true"]), " gpu-feature-discovery --version", t(["./build/gpu-feature-discovery", "--version"]))
PY
  for b in sysfs amdsmi; do
    echo "## --oneshot --backend=$b --trace-timing (3 runs)"
    for i in 1 2 3; do
      timeout -k 5 60 ./build/gpu-feature-discovery --oneshot --backend=$b --trace-timing -o $out/gfd 2>&1 | grep -E "Timing" || exit 1
    done
  done
} > $out/oneshot_probe.txt 2>&1
cat $out/oneshot_probe.txt
