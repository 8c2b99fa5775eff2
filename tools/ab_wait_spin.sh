#!/bin/bash
# A/B: a thread waiting for a pool task another thread is finishing spins
# up to ~10 us before it sleeps (default) or sleeps at once
# (GFD_AB_NO_WAIT_SPIN=1, the switch removed once decided -
# profiles/wait_spin_ab_r6.txt); alternated, 5 pairs, bench.py's untraced
# value and the traced steps' facts.wait.  Usage (GPU box): tools/ab_wait_spin.sh [outdir]
set -o pipefail
out=gpurun_out/${1:-ab_wait_spin}
mkdir -p $out
for rep in 1 2 3 4 5; do
  for v in spin sleep; do
    if [ $v = sleep ]; then export GFD_AB_NO_WAIT_SPIN=1; else unset GFD_AB_NO_WAIT_SPIN; fi
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 2000 --warmup 200 --no-extras > $out/${v}_$rep.json 2>/dev/null ||
      { echo "bench $v $rep failed"; exit 1; }
    python3 -c "
import json; r=json.load(open('$out/${v}_$rep.json')); p=r['phases_p50_ms']
print('$v rep $rep: value %.4f p90 %.4f traced %.4f | sriov.self %s sriov(overlapped) %s label %s facts.wait %s' % (
  r['value'], r['p90_ms'], r['traced_p50_ms'], p.get('sriov.self'), p.get('sriov(overlapped)'), p.get('label'), p.get('facts.wait')))"
  done
done | tee $out/summary.txt
