#!/bin/bash
# The driver's headline (bench.py --steps 20 --warmup 5, in-process) for a
# few variants, alternated: an older tree staged under abtree/<name>/
# (bench.py, gpu_feature_discovery_amd/ with its _gfd .so, build/ daemon)
# and the current tree.  Round 4 also ran the current tree with an
# experiment switch (GFD_PREPARE_PER_JOB, since removed):
# profiles/headline_ab_r4.txt.  One JSON line per run: value and the write
# phases.
# Usage (GPU box): tools/headline_ab.sh [reps] [steps] [warmup]
set -o pipefail
reps=${1:-4}; steps=${2:-20}; warm=${3:-5}
out=gpurun_out/headline_ab; mkdir -p $out
run() {  # name dir env...
  local name=$1 dir=$2; shift 2
  (cd "$dir" && env "$@" timeout -k 10 120 python3 bench.py --steps $steps --warmup $warm --no-extras --cold-cycles 0 \
    2>/dev/null) | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_p50_ms']
print(json.dumps({'variant': '$name', 'value': d['value'], 'p90': d['p90_ms'], 'write': p.get('write'),
  'create': p.get('write.create'), 'rename': p.get('write.rename')}))"
}
for i in $(seq $reps); do
  for d in abtree/*/; do
    [ -d "$d" ] && { run "$(basename "$d")" "$d" X=1 || exit 1; }
  done
  run current . X=1 || exit 1
done
