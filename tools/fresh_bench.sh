#!/bin/bash
# The driver's bench command as a fresh box's first command, then the file-system probe.
# Usage (GPU box): tools/fresh_bench.sh NAME
set -o pipefail
out=gpurun_out/${1:-fresh_bench}
mkdir -p "$out"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" ||
  { echo "bench failed"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); p=d['phases_p50_ms']
print('bench value', d['value'], 'p90', d['p90_ms'], 'cold', d['cold_cycle']['p50_ms'], 'first', d['first_cycle_ms'],
      'job', d['oneshot_process_p50_ms'], 'write', p.get('write'), 'rename', p.get('write.rename'), 'n', d.get('phases_n'))"
timeout -k 10 60 python3 tools/fs_probe.py > "$out/fs_probe.jsonl" 2>&1 || { echo "fs probe failed"; exit 1; }
