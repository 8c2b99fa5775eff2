#!/bin/bash
# A/B: the ROCm version kept under a directory watch (default) or looked up
# by path every cycle (GFD_AB_NO_VERSION_WATCH=1, the switch removed once
# decided - profiles/version_watch_ab_r6.txt); alternated, 5 pairs, bench.py's untraced value and the traced
# steps' facts.runtime / facts.wait.  Usage (GPU box): tools/ab_version_watch.sh [outdir]
set -o pipefail
out=gpurun_out/${1:-ab_version_watch}
mkdir -p $out
for rep in 1 2 3 4 5; do
  for v in watch path; do
    if [ $v = path ]; then export GFD_AB_NO_VERSION_WATCH=1; else unset GFD_AB_NO_VERSION_WATCH; fi
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 2000 --warmup 200 --no-extras > $out/${v}_$rep.json 2>/dev/null ||
      { echo "bench $v $rep failed"; exit 1; }
    python3 -c "
import json; r=json.load(open('$out/${v}_$rep.json')); p=r['phases_p50_ms']
print('$v rep $rep: value %.4f p90 %.4f traced %.4f | facts(overlapped) %s facts.runtime %s facts.wait %s label %s' % (
  r['value'], r['p90_ms'], r['traced_p50_ms'], p.get('facts(overlapped)'), p.get('facts.runtime'), p.get('facts.wait'), p.get('label')))"
  done
done | tee $out/summary.txt
