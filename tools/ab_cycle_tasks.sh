#!/bin/bash
# A/B on one box: node facts + SR-IOV scan on one worker in sequence (seq,
# default) vs as two separate pool tasks (split).  Interleaved, twice.
set -o pipefail
out=gpurun_out/${1:-ab}
mkdir -p $out
for round in 1 2; do
  for mode in seq split; do
    GFD_CYCLE_TASKS=$mode timeout -k 10 300 python bench.py --steps 1000 --warmup 100 > $out/$mode.$round.json 2> $out/$mode.$round.err || { echo "bench $mode failed"; exit 1; }
    python3 -c "
import json,sys; r=json.load(open('$out/$mode.$round.json')); e=r['extras']
print('$mode round $round: bench p50 %.4f p90 %.4f | loop p50 %.4f p90 %.4f | facts %.4f sriov %.4f snapshot %.4f' % (r['value'], r['p90_ms'], e['daemon_loop']['p50_ms'], e['daemon_loop']['p90_ms'], e['phases_ms']['facts(overlapped)'], e['phases_ms']['sriov(overlapped)'], e['phases_ms']['amdsmi.snapshot']))"
  done
done | tee $out/ab.txt
