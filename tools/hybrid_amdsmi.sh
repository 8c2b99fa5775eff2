#!/bin/bash
# 1/2/4/8-GPU curve of the amd-smi backend over the host's real GPUs: the fake
# libamd_smi (tests/fake_amdsmi) reports the host's 8 MI355X at their real PCI
# addresses, so the backend's per-GPU work - the snapshot, one lane per GPU,
# the attribute preads of each GPU's live amdgpu attributes (partition modes,
# VRAM, xGMI links, capabilities, product name) - runs over the real driver
# of up to 8 GPUs, while the library's own calls cost what the fake charges:
# nothing (latency 0) or LAT us per device query (e.g. 1).  A one-GPU box's
# amd-smi sees only its own GPU; this is as close to the 8-GPU amd-smi case
# as it can get.  Back to back (bench.py) and cycles 1 s apart (cold_cycle.py).
# Usage (GPU box): tools/hybrid_amdsmi.sh [outdir] [LAT]
set -o pipefail
out=gpurun_out/${1:-hybrid_amdsmi}
lat=${2:-0}
mkdir -p $out
spec=$(python3 tools/hybrid_amdsmi_spec.py "$lat") || exit 1
n=$(echo "$spec" | tr '|' '\n' | grep -c '^bdf=')
echo "GPUs reported by the fake library at the host's addresses: $n (device query latency ${lat} us)"
export GFD_AMDSMI_LIBRARY=$PWD/build/libfake_amdsmi.so GFD_FAKE_AMDSMI_SPEC="$spec"
for g in 1 2 4 8; do
  [ $g -le $n ] || break
  timeout -k 10 300 python3 bench.py --gpus $g --steps 2000 --warmup 200 --backend amdsmi --no-extras \
    > $out/amdsmi_$g.json 2> $out/amdsmi_$g.err || { echo "bench $g failed"; tail -5 $out/amdsmi_$g.err; exit 1; }
  timeout -k 10 120 python3 tools/cold_cycle.py --backend amdsmi --visible-devices 0-$((g - 1)) \
    --interval 1s --cycles 10 > $out/cold_$g.json 2> $out/cold_$g.err ||
    { echo "cold $g failed"; tail -5 $out/cold_$g.err; exit 1; }
  python3 -c "
import json; r=json.load(open('$out/amdsmi_$g.json'))
c=[json.loads(l) for l in open('$out/cold_$g.json') if l.startswith('{')][0]
p=r['phases_p50_ms']
q=c['phases_p50_ms']
lanes=lambda p: ' '.join('%s %s' % (k.split('.')[-1], p.get(k)) for k in ('amdsmi.lanes.handoff', 'amdsmi.lanes.last_start', 'amdsmi.lanes.max_gpu', 'amdsmi.lanes.caller_gpus(count_as_ms)') if k in p)
print('%d GPU(s): back to back p50 %.4f ms p90 %.4f ms | 1 s apart p50 %.3f ms | labels_ok=%s count=%s | enumerate %s amdsmi.gpus %s label %s write %s' % (
  $g, r['value'], r['p90_ms'], c['p50_ms'], r['labels_ok'], r['n_gpus'], p.get('enumerate'), p.get('amdsmi.gpus'),
  p.get('label'), p.get('write')))
if $g > 1:
  print('    lanes back to back: %s | 1 s apart: %s (amdsmi.gpus %s)' % (lanes(p), lanes(q), q.get('amdsmi.gpus')))"
done | tee $out/curve.txt
