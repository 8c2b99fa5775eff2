#!/bin/bash
# Labeling latency while the GPU is busy, as on a node running a training
# job: the headline bench (back to back) and the daemon at 1 s cadence, first
# with the GPU idle, then with a PyTorch bf16 GEMM loop keeping it at full
# load (a separate process, stopped by its PID), then idle again (the order
# matters: a fresh box's first run is slow).  Every step is time-limited.
# Usage (GPU box): tools/busy_gpu.sh [outdir-name]
set -o pipefail
out=gpurun_out/${1:-busy}
mkdir -p "$out"
measure() {
  timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-extras > "$out/bench_$1.json" 2> "$out/bench_$1.err" ||
    { echo "bench $1 failed"; return 1; }
  timeout -k 10 60 python tools/cold_cycle.py --interval 1s --cycles 15 > "$out/cold_$1.json" 2> "$out/cold_$1.err" ||
    { echo "cold $1 failed"; return 1; }
  python3 -c "
import json; r=json.load(open('$out/bench_$1.json')); c=json.load(open('$out/cold_$1.json'))
print('%-5s back to back p50 %.4f ms p90 %.4f ms | 1 s apart p50 %.3f ms p90 %.3f ms | labels_ok=%s' % (
  '$1', r['value'], r['p90_ms'], c['p50_ms'], c['p90_ms'], r['labels_ok']))"
}
measure idle || exit 1
timeout -k 10 150 python -u -c "
import time, torch
a = torch.randn(8192, 8192, device='cuda', dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device='cuda', dtype=torch.bfloat16)
torch.cuda.synchronize()
t0, n = time.time(), 0
while time.time() - t0 < 120:
    for _ in range(20):
        c = a @ b
    torch.cuda.synchronize()
    n += 20
    if n % 2000 == 0:
        print('load: %d GEMMs, %.0f TFLOP/s' % (n, 2 * 8192**3 * n / (time.time() - t0) / 1e12), flush=True)
" > "$out/load.log" 2>&1 &
load=$!
sleep 15
kill -0 $load 2>/dev/null || { echo "load process ended early"; tail -5 "$out/load.log"; exit 1; }
measure busy; rc=$?
kill $load 2>/dev/null; wait $load 2>/dev/null
tail -2 "$out/load.log"
[ $rc -eq 0 ] || exit $rc
sleep 5
measure idle2
