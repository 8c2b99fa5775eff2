#!/bin/bash
# A/B: the 8-GPU hybrid snapshot with every value session-cached, run inline
# on the cycle thread (GFD_INLINE_CACHED=1, default) or one lane per GPU
# (=0); back to back (bench.py) and 1 s apart (tools/cold_cycle.py).
# (Its experiment switch was removed from the daemon once the A/B decided - see
# profiles/hybrid_amdsmi_scaling_r6.txt; the script records how those numbers were taken.)
set -o pipefail
out=gpurun_out/${1:-ab_inline}
mkdir -p $out
spec=$(python3 tools/hybrid_amdsmi_spec.py 0) || exit 1
export GFD_AMDSMI_LIBRARY=$PWD/build/libfake_amdsmi.so GFD_FAKE_AMDSMI_SPEC="$spec"
for rep in 1 2 3; do
  for v in 1 0; do
    GFD_INLINE_CACHED=$v timeout -k 10 120 python3 bench.py --gpus 8 --steps 2000 --warmup 200 --backend amdsmi \
      --no-extras > $out/b2b_${v}_$rep.json 2>/dev/null || exit 1
  done
done
timeout -k 10 400 python3 tools/cold_cycle.py --backend amdsmi --visible-devices 0-7 --interval 1s --cycles 10 \
  --variants "GFD_INLINE_CACHED=1,GFD_INLINE_CACHED=0" --reps 3 > $out/cold.jsonl 2>&1 || exit 1
python3 - "$out" <<'PY'
import json, sys, statistics
out = sys.argv[1]
for v in (1, 0):
    xs = [json.loads([l for l in open(f"{out}/b2b_{v}_{r}.json") if l.startswith("{")][-1]) for r in (1, 2, 3)]
    print(f"inline_cached={v} back to back 8 GPUs: {[x['value'] for x in xs]} amdsmi.gpus "
          f"{[x['phases_p50_ms'].get('amdsmi.gpus') for x in xs]} enumerate {[x['phases_p50_ms'].get('enumerate') for x in xs]}")
for line in open(f"{out}/cold.jsonl"):
    if line.startswith('{"summary"'):
        print(line.strip())
for line in open(f"{out}/cold.jsonl"):
    if line.startswith('{"variant"'):
        r = json.loads(line)
        print(r["variant"], r["rep"], "p50", r["p50_ms"], "enumerate", r["phases_p50_ms"].get("enumerate"),
              "amdsmi.gpus", r["phases_p50_ms"].get("amdsmi.gpus"))
PY
