#!/bin/bash
# A/B of WorkerPool::prewake (GFD_EXP_PREWAKE=off disables it) on the amd-smi
# backend over the host's real GPUs (tools/hybrid_amdsmi_spec.py), alternated:
# back to back (bench.py, 2000 steps) and cycles 1 s apart (cold_cycle.py),
# at 2 and 8 GPUs.  Needs the experiment build of commit bca62c4 (prewake was
# not kept: docs/ROUND5.md).  Usage (GPU box): tools/prewake_ab.sh [outdir] [reps]
set -o pipefail
out=gpurun_out/${1:-prewake_ab}; reps=${2:-3}
mkdir -p $out
spec=$(python3 tools/hybrid_amdsmi_spec.py 0) || exit 1
export GFD_AMDSMI_LIBRARY=$PWD/build/libfake_amdsmi.so GFD_FAKE_AMDSMI_SPEC="$spec"
for g in 2 8; do
  for r in $(seq 1 $reps); do
    for v in fan direct off; do
      e="GFD_EXP_PREWAKE=$v"
      env $e timeout -k 10 300 python3 bench.py --gpus $g --steps 2000 --warmup 200 --backend amdsmi --no-extras \
        > $out/b_${g}_${v}_$r.json 2> $out/b_${g}_${v}_$r.err || { echo "bench $g $v failed"; tail -3 $out/b_${g}_${v}_$r.err; exit 1; }
      python3 -c "
import json; r=json.load(open('$out/b_${g}_${v}_$r.json')); p=r['phases_p50_ms']
print(json.dumps({'gpus': $g, 'prewake': '$v', 'rep': $r, 'value': r['value'], 'p90': r['p90_ms'], 'gpus_ms': p.get('amdsmi.gpus'),
                  'enumerate': p.get('enumerate'), 'placement': p.get('placement'), 'ok': r['labels_ok']}))"
    done
  done
  timeout -k 10 400 python3 tools/cold_cycle.py --backend amdsmi --visible-devices 0-$((g - 1)) --interval 1s \
    --cycles 10 --reps $reps --variants "GFD_EXP_PREWAKE=fan --cpu-affinity=follow,GFD_EXP_PREWAKE=direct --cpu-affinity=follow,GFD_EXP_PREWAKE=off --cpu-affinity=follow" \
    > $out/cold_$g.jsonl 2> $out/cold_$g.err || { echo "cold $g failed"; tail -3 $out/cold_$g.err; exit 1; }
  python3 -c "
import json, statistics
runs = [json.loads(l) for l in open('$out/cold_$g.jsonl') if l.startswith('{') and 'summary' not in l]
for v in dict.fromkeys(r['variant'] for r in runs):
    rs = [r for r in runs if r['variant'] == v]
    med = lambda k: round(statistics.median(r['phases_p50_ms'].get(k, 0) for r in rs), 4)
    print(json.dumps({'gpus': $g, 'cold_variant': v, 'p50s': [r['p50_ms'] for r in rs],
                      'p50': round(statistics.median(r['p50_ms'] for r in rs), 4), 'gpus_ms': med('amdsmi.gpus'),
                      'placement': med('placement')}))"
done | tee $out/summary.txt
