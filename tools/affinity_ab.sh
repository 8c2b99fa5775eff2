#!/bin/bash
# Same-box A/B of the daemon's CPU placement policies, hot bench p50 (500
# back-to-back cycles): L3-domain pinning (GFD_CPU_AFFINITY, default on) x
# the pool's adaptive spin (GFD_POOL_SPIN_US, default 200), alternated.
# Usage (GPU box): tools/affinity_ab.sh > gpurun_out/affinity_ab.txt
cpu=$(python3 -c "import os; print(sorted(os.sched_getaffinity(0))[0])")
echo "allowed CPUs: $(python3 -c "import os; print(len(os.sched_getaffinity(0)))"); L3 domain of cpu$cpu: $(cat /sys/devices/system/cpu/cpu$cpu/cache/index3/shared_cpu_list)"
lscpu | grep -E "Model name|Socket|NUMA node\(s\)|L3" || true
for rep in 1 2 3; do
  for aff in none l3; do
    for spin in 0 200; do
      v=$(GFD_CPU_AFFINITY=$aff GFD_POOL_SPIN_US=$spin timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-extras 2>/dev/null |
          python3 -c "import json,sys; r=json.loads(sys.stdin.read()); p=r['phases_p50_ms']; print(r['value'], r['p90_ms'], p.get('label'), p.get('amdsmi.gpus'), p.get('write'))")
      echo "rep $rep affinity=$aff spin=${spin}us: hot p50 p90 label amdsmi.gpus write = $v"
    done
  done
done
