#!/bin/bash
# What phase tracing costs a back-to-back cycle: bench.py reports the timed
# steps untraced (value) and the same K steps traced right after
# (traced_p50_ms); five runs in fresh processes on one box, then the
# driver's own command.  Usage (GPU box): tools/trace_ab.sh [outdir]
set -o pipefail
out=gpurun_out/${1:-trace_ab}
mkdir -p "$out"
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 2000 --warmup 200 --no-extras > "$out/run_$i.json" 2> "$out/run_$i.err" ||
    { echo "run $i failed"; tail -5 "$out/run_$i.err"; exit 1; }
  python3 -c "
import json; r=json.load(open('$out/run_$i.json'))
print('run $i: untraced p50 %.4f p90 %.4f | traced p50 %.4f | labels_ok %s' % (r['value'], r['p90_ms'], r['traced_p50_ms'], r['labels_ok']))"
done | tee "$out/summary.txt"
