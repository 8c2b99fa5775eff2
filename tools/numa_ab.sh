#!/bin/bash
# Same-box A/B: the hot bench pinned to an L3 domain (CCD) on the GPU's own
# socket vs one on the other socket (GFD_CPU_AFFINITY=none + taskset).
# Usage (GPU box): tools/numa_ab.sh > gpurun_out/numa_ab.txt
bdf=$(basename $(readlink -f /sys/class/drm/renderD*/device | head -1))
node=$(cat /sys/bus/pci/devices/$bdf/numa_node)
local_list=$(cat /sys/bus/pci/devices/$bdf/local_cpulist)
echo "GPU $bdf numa_node $node local CPUs $local_list"
first_local=$(python3 -c "print(int('$local_list'.split(',')[0].split('-')[0]))")
l3_local=$(cat /sys/devices/system/cpu/cpu$first_local/cache/index3/shared_cpu_list)
remote=$(python3 -c "
import glob
loc=set()
for part in '$local_list'.split(','):
    a,_,b=part.partition('-'); loc.update(range(int(a), int(b or a)+1))
print(min(c for c in range(512) if c not in loc and __import__('os').path.exists(f'/sys/devices/system/cpu/cpu{c}')))")
l3_remote=$(cat /sys/devices/system/cpu/cpu$remote/cache/index3/shared_cpu_list)
echo "local L3 $l3_local, remote L3 $l3_remote"
for rep in 1 2 3; do
  for where in local remote; do
    if [ $where = local ]; then l=$l3_local; else l=$l3_remote; fi
    v=$(GFD_CPU_AFFINITY=none taskset -c $l timeout -k 10 120 python bench.py --steps 500 --warmup 50 --no-extras 2>/dev/null |
        python3 -c "import json,sys; r=json.loads(sys.stdin.read()); p=r['phases_p50_ms']; print(r['value'], r['p90_ms'], p.get('label'), p.get('amdsmi.gpus'), p.get('write'))")
    echo "rep $rep $where: hot p50 p90 label amdsmi.gpus write = $v"
  done
done
