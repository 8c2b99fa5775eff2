#!/bin/bash
# A fresh box's pass in the driver's order: the driver's bench command first
# (the regime BENCH_rNN records), then the file-system probe, the GPU test
# suite and the smoke entry point.  Every step is time-limited and the first
# failure ends the pass.
# Usage (GPU box): tools/fresh_pass.sh [outdir-name]
set -o pipefail
out=gpurun_out/${1:-fresh_pass}
mkdir -p "$out"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" ||
  { echo "bench failed"; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); p=d['phases_p50_ms']
print('bench value', d['value'], 'p90', d['p90_ms'], 'cold', d['cold_cycle']['p50_ms'], 'first', d['first_cycle_ms'],
      'job', d['oneshot_process_p50_ms'], 'write', p.get('write'), 'rename', p.get('write.rename'), 'n', d.get('phases_n'))"
timeout -k 10 60 python3 tools/fs_probe.py > "$out/fs_probe.jsonl" 2>&1 || { echo "fs probe failed"; exit 1; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$out/pytest_gpu.txt" 2>&1; rc=$?
tail -3 "$out/pytest_gpu.txt"
[ $rc -eq 0 ] || { echo "pytest -m gpu failed rc=$rc"; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || { echo "smoke failed"; exit 1; }
tail -2 "$out/smoke.txt"
echo "pass ok: $out"
