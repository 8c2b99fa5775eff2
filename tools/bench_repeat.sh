#!/bin/bash
# The headline bench repeated on one box (no extras): within-box spread.
set -o pipefail
out=gpurun_out/${1:-repeat}
mkdir -p $out
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-extras > $out/b$i.json 2> $out/b$i.err || { echo "bench $i failed"; exit 1; }
  python3 -c "import json; r=json.load(open('$out/b$i.json')); print('run $i: p50 %.4f ms p90 %.4f ms mean %.4f ms' % (r['value'], r['p90_ms'], r['mean_ms']))"
done | tee $out/repeat.txt
