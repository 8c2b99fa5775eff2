#!/bin/bash
# Generic A/B of one environment setting on the bench, alternated on one box:
# the default vs VAR=value, REPS times each; prints the hot and cold cycle
# with the write's sub-phases (write.take/create, write.data, write.rename).
# Usage (GPU box): tools/env_ab.sh <outdir-name> <reps> VAR=value [bench args...]
set -o pipefail
out=gpurun_out/${1:?outdir}
reps=${2:?reps}
setting=${3:?VAR=value}
shift 3
var=${setting%%=*}
val=${setting#*=}
mkdir -p "$out"
for r in $(seq 1 "$reps"); do
  for mode in default "$setting"; do
    tag=$([ "$mode" = default ] && echo default || echo alt)
    if [ "$mode" = default ]; then unset "$var"; else export "$var=$val"; fi
    timeout -k 10 300 python bench.py --steps 2000 --warmup 200 "$@" > "$out/${tag}_$r.json" 2> "$out/${tag}_$r.err" \
      || { echo "bench failed"; tail -5 "$out/${tag}_$r.err"; exit 1; }
    python3 - "$out/${tag}_$r.json" "$r" "$mode" <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); c = r.get("cold_cycle") or {}
def w(ph):
    return " ".join(f"{k[6:]}={v * 1000:.1f}" for k, v in sorted(ph.items()) if k.startswith("write."))
print(f"rep {sys.argv[2]} {sys.argv[3]:28s}: hot p50 {r['value']:.4f} p90 {r['p90_ms']:.4f} ms (write {r['phases_p50_ms'].get('write', 0) * 1000:.1f} us: {w(r['phases_p50_ms'])})"
      f" | cold p50 {c.get('p50_ms', 0):.3f} ms (write {c.get('phases_p50_ms', {}).get('write', 0) * 1000:.0f} us: {w(c.get('phases_p50_ms', {}))})"
      f" | daemon loop {r['extras'].get('daemon_loop', {}).get('p50_ms', 0):.4f}")
PY
  done
done | tee "$out/ab.txt"
