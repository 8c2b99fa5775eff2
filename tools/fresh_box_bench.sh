#!/bin/bash
# The bench on a freshly started box, then after sync, then 45 s later: is
# a slow first run the file system settling?  (profiles/busy_gpu_r3.txt)
set -o pipefail
mkdir -p gpurun_out/fresh
b() { timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-extras > gpurun_out/fresh/$1.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/fresh/$1.json')); p=d['phases_p50_ms']
print('%-8s p50 %.4f p90 %.4f write.rename %.4f write.create %s' % ('$1', d['value'], d['p90_ms'], p.get('write.rename',0), p.get('write.create')))"; }
grep -E "Dirty|Writeback:" /proc/meminfo | tr '\n' ' '; echo
b first && grep -E "Dirty|Writeback:" /proc/meminfo | tr '\n' ' ' && echo && timeout 60 sync && echo synced && b after_sync && sleep 45 && b later
