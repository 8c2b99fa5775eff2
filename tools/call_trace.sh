#!/bin/bash
# Per-call amd-smi latency inside the daemon loop (100 cycles).
mkdir -p gpurun_out/ct
GFD_AMDSMI_CALL_TRACE=1 timeout -k 5 20 ./build/gpu-feature-discovery --sleep-interval=5ms --trace-timing -o gpurun_out/ct/gfd > gpurun_out/ct/loop.log 2>&1
grep Timing gpurun_out/ct/loop.log | tail -3
