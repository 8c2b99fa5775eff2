#!/bin/bash
# The headline bench (no extras) under each write mode on one box, with the
# write's sub-phases, plus what /tmp (the bench's output directory) is.
# Usage (GPU box): tools/write_modes_probe.sh [outdir-name] [reps]
set -o pipefail
out=gpurun_out/${1:-write_modes}
mkdir -p "$out"
{
  echo "# /tmp: $(stat -f -c %T /tmp)"
  for r in $(seq 1 "${2:-2}"); do
    for mode in X=1 GFD_WRITE_PREPARE=never GFD_WRITE_PREALLOC=never "GFD_WRITE_PREPARE=never GFD_WRITE_PREALLOC=never"; do
      tag=$(echo "$mode" | tr ' =' '__')
      env $mode timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-extras > "$out/$tag_$r.json" 2> "$out/$tag_$r.err" \
        || { echo "bench failed"; tail -5 "$out/$tag_$r.err"; exit 1; }
      python3 - "$out/$tag_$r.json" "$mode" <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); p = r["phases_p50_ms"]
print(f"{sys.argv[2]:50s}: p50 {r['value']:.4f} p90 {r['p90_ms']:.4f} | "
      + " ".join(f"{k}={v * 1000:.1f}" for k, v in sorted(p.items()) if k.startswith("write")))
PY
    done
  done
} | tee "$out/probe.txt"
