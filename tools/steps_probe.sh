#!/bin/bash
# Headline bench at several --steps/--warmup settings (no extras), with the
# write's sub-phases: does the prepared temporary file keep up?
# Usage (GPU box): tools/steps_probe.sh [outdir-name] [reps]
set -o pipefail
out=gpurun_out/${1:-steps_probe}
mkdir -p "$out"
for r in $(seq 1 "${2:-2}"); do
  for sw in "200 20" "200 200" "2000 200" "20 5"; do
    set -- $sw
    timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-extras > "$out/s$1_w$2_$r.json" 2> "$out/s$1_w$2_$r.err" \
      || { echo "bench failed"; tail -5 "$out/s$1_w$2_$r.err"; exit 1; }
    python3 - "$out/s$1_w$2_$r.json" "$1" "$2" <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); p = r["phases_p50_ms"]
print(f"steps {sys.argv[2]:>4} warmup {sys.argv[3]:>3}: p50 {r['value']:.4f} p90 {r['p90_ms']:.4f} ms/step {r['ms_per_step']:.4f} | "
      + " ".join(f"{k}={v * 1000:.1f}" for k, v in sorted(p.items()) if k.startswith("write") or k in ("enumerate", "label")))
PY
  done
done | tee "$out/probe.txt"
