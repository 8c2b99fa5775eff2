#!/bin/bash
# Where a oneshot (Job-mode) process spends its time, per backend: wall time
# of the whole process (as bench.py's oneshot_process measures it), the
# daemon's own phase trace, dynamic-linker statistics, and - when strace is
# installed - a timestamped syscall trace of one sysfs run.
# Usage (GPU box): tools/oneshot_breakdown.sh [outdir-name]
set -o pipefail
out=gpurun_out/${1:-oneshot_breakdown}
mkdir -p "$out"
bin=./build/gpu-feature-discovery
{
  python3 - "$bin" "$out" <<'PY'
import statistics, subprocess, sys, time
binary, out = sys.argv[1], sys.argv[2]
sys.path.insert(0, ".")
from gpu_feature_discovery_amd.utils.proc import spawn_wait_ms  # blocking waitpid, no polling quantisation
def wall(cmd, n=30, env=None):
    xs = sorted(spawn_wait_ms(cmd, timeout=60, env=env) for _ in range(n))
    return f"p50 {statistics.median(xs):8.3f} ms  p90 {xs[int(0.9 * (len(xs) - 1))]:8.3f} ms"
o = ["--oneshot", f"--output-file={out}/gfd"]
print("## process wall time (30 runs each)")
for name, cmd in [("/bin/true", ["/bin/true"]),
                  ("--version", [binary, "--version"]),
                  ("oneshot null", [binary, *o, "--backend=null"]),
                  ("oneshot sysfs", [binary, *o, "--backend=sysfs"]),
                  ("oneshot auto", [binary, *o, "--backend=auto"]),
                  ("oneshot amdsmi", [binary, *o, "--backend=amdsmi"])]:
    print(f"{name:16s} {wall(cmd, 10 if 'amdsmi' in name else 30)}")
PY
  for b in null sysfs auto amdsmi; do
    echo "## --oneshot --backend=$b --trace-timing"
    timeout -k 5 60 "$bin" --oneshot --backend=$b --trace-timing -o "$out/gfd" 2>&1 | grep -iE "timing:|Using|Detected" || exit 1
  done
  echo "## LD_DEBUG=statistics --version"
  LD_DEBUG=statistics timeout -k 5 30 "$bin" --version 2>&1 | grep -E "time|relocations" | head -12
  if command -v strace > /dev/null; then
    echo "## strace -f -r --oneshot --backend=sysfs (relative timestamps; syscalls slower than 100 us or around gaps)"
    timeout -k 5 60 strace -f -r -o "$out/strace_sysfs.txt" "$bin" --oneshot --backend=sysfs -o "$out/gfd" > /dev/null 2>&1 || true
    wc -l < "$out/strace_sysfs.txt"
    awk '$2+0 > 0.0001 || $3+0 > 0.0001' "$out/strace_sysfs.txt" | head -80
    echo "## syscall counts"
    timeout -k 5 60 strace -f -c -o "$out/strace_c.txt" "$bin" --oneshot --backend=sysfs -o "$out/gfd" > /dev/null 2>&1 || true
    head -40 "$out/strace_c.txt"
  else
    echo "## strace not installed"
  fi
} > "$out/breakdown.txt" 2>&1
rc=$?
cat "$out/breakdown.txt"
exit $rc
