#!/bin/bash
# Same-box A/B of the worker pool's adaptive idle spin (GFD_POOL_SPIN_US bound, 0 = off): hot bench
# p50 (500 back-to-back cycles) and the daemon's cycles 1 s apart, alternated.
# Usage (GPU box): tools/pool_spin_ab.sh > gpurun_out/pool_spin_ab.txt
for rep in 1 2 3 4; do
  for us in 0 200; do
    v=$(GFD_POOL_SPIN_US=$us timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-extras 2>/dev/null |
        python -c "import json,sys; r=json.loads(sys.stdin.read()); p=r['phases_p50_ms']; print(r['value'], r['p90_ms'], p.get('label'), p.get('amdsmi.gpus'), p.get('write'))")
    echo "rep $rep spin ${us}us: hot p50 p90 label amdsmi.gpus write = $v"
  done
done
for us in 0 200; do
  v=$(GFD_POOL_SPIN_US=$us timeout -k 10 120 python - <<'PY'
import os, sys
sys.path.insert(0, os.getcwd())
import bench, gpu_feature_discovery_amd as gfd
r = bench._daemon_loop(str(gfd.binary_path()), ["--backend=auto", "--output-file=/tmp/gfd-spin-ab"], 10, interval="1s")
print(r["p50_ms"], r["p90_ms"], r["phases_p50_ms"].get("write"))
PY
)
  echo "spin ${us}us: cold cycle (1 s apart) p50 p90 write = $v"
done
