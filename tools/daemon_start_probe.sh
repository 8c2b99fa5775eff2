#!/bin/bash
# Daemon start-up as deployed (--backend=auto): backend selection (library
# probing), the first cycle (KFD while amd-smi initialises in the
# background), the switch, and the process timeline printed at exit.
# Usage (GPU box): tools/daemon_start_probe.sh [outdir-name]
out=gpurun_out/${1:-daemon_start}
mkdir -p "$out"
for i in 1 2 3; do
  timeout -k 5 30 ./build/gpu-feature-discovery --trace-timing --sleep-interval=50ms -o "$out/gfd" > /dev/null 2> "$out/run$i.err" &
  pid=$!
  sleep 1
  kill -TERM $pid
  wait $pid
  grep -iE "timing:|Detected|Using|Initializing" "$out/run$i.err" | head -12
done
