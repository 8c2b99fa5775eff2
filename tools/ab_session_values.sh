#!/bin/bash
# A/B of values kept per amd-smi session (GFD_SESSION_VALUES=1) against reading them every cycle.
# (Its experiment switch was removed from the daemon once the A/B decided - see
# profiles/hybrid_amdsmi_scaling_r6.txt; the script records how those numbers were taken.)
set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 300 python3 tools/variants_ab.py --variant base= --variant sv=GFD_SESSION_VALUES=1 --reps 5 --modes headline,cold --cold-cycles 8 > gpurun_out/r6e/ab.jsonl 2>&1 || exit 1
spec=$(python3 tools/hybrid_amdsmi_spec.py 0) || exit 1
for rep in 1 2 3; do
 for v in 0 1; do
  GFD_SESSION_VALUES=$v GFD_AMDSMI_LIBRARY=$PWD/build/libfake_amdsmi.so GFD_FAKE_AMDSMI_SPEC="$spec" timeout -k 10 120 python3 bench.py --gpus 8 --steps 2000 --warmup 200 --backend amdsmi --no-extras > gpurun_out/r6e/h8_${v}_$rep.json 2>/dev/null || exit 1
  GFD_SESSION_VALUES=$v GFD_AMDSMI_LIBRARY=$PWD/build/libfake_amdsmi.so GFD_FAKE_AMDSMI_SPEC="$spec" timeout -k 10 120 python3 bench.py --gpus 1 --steps 2000 --warmup 200 --backend amdsmi --no-extras > gpurun_out/r6e/h1_${v}_$rep.json 2>/dev/null || exit 1
 done
done
GFD_AMDSMI_CALL_TRACE=1 timeout -k 10 60 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-extras --cold-cycles 0 > gpurun_out/r6e/calltrace.json 2>/dev/null
echo done
