#!/bin/bash
# Lanes A/B for the per-GPU work of a cycle on the host's 8 real GPUs
# (KFD-sysfs backend over tools/hybrid_root.py), back to back and in the
# daemon loop (2 ms sleep between cycles).
set -o pipefail
out=gpurun_out/${1:-lanes}
mkdir -p $out
root=$(mktemp -d /tmp/gfd-hybrid-XXXXXX)
n=$(python3 tools/hybrid_root.py $root) || exit 1
for lanes in 1 2 4 8 auto; do
  for g in ${GPUS:-1 8}; do
    [ $g -le $n ] || continue
    if [ $lanes = auto ]; then unset GFD_GPU_LANES; else export GFD_GPU_LANES=$lanes; fi
    timeout -k 10 300 python bench.py --gpus $g --steps 2000 --warmup 200 --backend sysfs --sysfs-root $root --cold-cycles 0 \
      > $out/l${lanes}_g$g.json 2> $out/l${lanes}_g$g.err || { echo "bench failed"; tail -5 $out/l${lanes}_g$g.err; exit 1; }
    python3 -c "
import json; r=json.load(open('$out/l${lanes}_g$g.json')); e=r['extras']
print('lanes=$lanes gpus=$g: bench p50 %.4f ms (gpus phase %.4f) | daemon loop p50 %.4f p90 %.4f' % (r['value'], r['phases_p50_ms'].get('sysfs.gpus', 0), e['daemon_loop']['p50_ms'], e['daemon_loop']['p90_ms']))"
  done
done | tee $out/lanes.txt
