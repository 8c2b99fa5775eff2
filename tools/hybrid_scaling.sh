#!/bin/bash
# 1/2/4/8-GPU curve of the KFD-sysfs backend over the host's real GPUs
# (tools/hybrid_root.py): live amdgpu attribute reads of up to 8 MI355X,
# back to back (bench.py) and as deployed, cycles 1 s apart (cold_cycle.py).
set -o pipefail
out=gpurun_out/${1:-hybrid}
mkdir -p $out
root=$(mktemp -d /tmp/gfd-hybrid-XXXXXX)
n=$(python3 tools/hybrid_root.py $root) || exit 1
echo "GPUs in the hybrid root: $n"
for g in 1 2 4 8; do
  [ $g -le $n ] || break
  timeout -k 10 300 python bench.py --gpus $g --steps 2000 --warmup 200 --backend sysfs \
    --sysfs-root $root --no-extras > $out/sysfs_$g.json 2> $out/sysfs_$g.err ||
    { echo "bench $g failed"; tail -5 $out/sysfs_$g.err; exit 1; }
  timeout -k 10 120 python tools/cold_cycle.py --backend sysfs --sysfs-root $root --visible-devices 0-$((g - 1)) \
    --interval 1s --cycles 10 > $out/cold_$g.json 2> $out/cold_$g.err ||
    { echo "cold $g failed"; tail -5 $out/cold_$g.err; exit 1; }
  python3 -c "
import json; r=json.load(open('$out/sysfs_$g.json'))
c=[json.loads(l) for l in open('$out/cold_$g.json') if l.startswith('{')][0]  # the run's line
print('%d GPU(s): back to back p50 %.4f ms p90 %.4f ms | 1 s apart p50 %.3f ms | labels_ok=%s count=%s | enumerate %s ms' % (
  $g, r['value'], r['p90_ms'], c['p50_ms'], r['labels_ok'], r['n_gpus'], r['phases_p50_ms'].get('enumerate')))"
done | tee $out/curve.txt
