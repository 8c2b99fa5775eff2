#!/bin/bash
# A/B of the 8-GPU hybrid snapshot (fake amd-smi at the host's 8 real GPUs):
# lanes (GFD_GPU_LANES) x session values (GFD_SESSION_VALUES), alternated.
# (Its experiment switch was removed from the daemon once the A/B decided - see
# profiles/hybrid_amdsmi_scaling_r6.txt; the script records how those numbers were taken.)
set -o pipefail
out=gpurun_out/${1:-ab_lanes}
mkdir -p $out
spec=$(python3 tools/hybrid_amdsmi_spec.py 0) || exit 1
export GFD_AMDSMI_LIBRARY=$PWD/build/libfake_amdsmi.so GFD_FAKE_AMDSMI_SPEC="$spec"
for rep in 1 2 3; do
  for lanes in 8 4 2; do
    for sv in 0 1; do
      GFD_GPU_LANES=$lanes GFD_SESSION_VALUES=$sv timeout -k 10 120 python3 bench.py --gpus 8 --steps 2000 --warmup 200 \
        --backend amdsmi --no-extras > $out/l${lanes}_sv${sv}_$rep.json 2>/dev/null || exit 1
    done
  done
done
python3 - "$out" <<'PY'
import json, sys, statistics
out = sys.argv[1]
for lanes in (8, 4, 2):
    for sv in (0, 1):
        xs = [json.loads([l for l in open(f"{out}/l{lanes}_sv{sv}_{r}.json") if l.startswith("{")][-1]) for r in (1, 2, 3)]
        p = [x["phases_p50_ms"] for x in xs]
        print(f"lanes {lanes} session_values {sv}: p50 {[x['value'] for x in xs]} median {statistics.median(x['value'] for x in xs)}"
              f" | amdsmi.gpus {[q.get('amdsmi.gpus') for q in p]} handoff {[q.get('amdsmi.lanes.handoff') for q in p]}"
              f" last_start {[q.get('amdsmi.lanes.last_start') for q in p]} max_gpu {[q.get('amdsmi.lanes.max_gpu') for q in p]}"
              f" enumerate {[q.get('enumerate') for q in p]}")
PY
