#!/bin/bash
# 1/2/4/8-GPU curve of the KFD-sysfs backend over the host's real GPUs
# (tools/hybrid_root.py): live amdgpu attribute reads of up to 8 MI355X.
set -o pipefail
out=gpurun_out/${1:-hybrid}
mkdir -p $out
root=$(mktemp -d /tmp/gfd-hybrid-XXXXXX)
n=$(python3 tools/hybrid_root.py $root) || exit 1
echo "GPUs in the hybrid root: $n"
# GFD_POOL_SPIN_US: the pool's adaptive idle spin off (0) and on (default).
for spin in 0 200; do
  for g in 1 2 4 8; do
    [ $g -le $n ] || break
    GFD_POOL_SPIN_US=$spin timeout -k 10 300 python bench.py --gpus $g --steps 2000 --warmup 200 --backend sysfs \
      --sysfs-root $root --no-extras > $out/sysfs_$g.json 2> $out/sysfs_$g.err ||
      { echo "bench $g failed"; tail -5 $out/sysfs_$g.err; exit 1; }
    python3 -c "
import json; r=json.load(open('$out/sysfs_$g.json'))
print('spin %sus %d GPU(s): p50 %.4f ms p90 %.4f ms labels_ok=%s count=%s | %s' % ('$spin', $g, r['value'], r['p90_ms'], r['labels_ok'], r['n_gpus'], ' '.join('%s=%.4f' % kv for kv in r['phases_p50_ms'].items())))"
  done
done | tee $out/curve.txt
