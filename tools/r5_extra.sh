#!/bin/bash
# Round-5 extra GPU measurements on the final code: the 1/2/4/8-GPU curve over
# the host's real GPUs (KFD-sysfs backend, tools/hybrid_scaling.sh), the Job
# process breakdown, and a longer soak of the loop writer (amd-smi backend).
set -o pipefail
timeout -k 10 600 bash tools/hybrid_scaling.sh r5f_hybrid || { echo "hybrid failed"; exit 1; }
timeout -k 10 300 bash tools/oneshot_breakdown.sh r5f_job > /dev/null || { echo "breakdown failed"; exit 1; }
GFD_SOAK_SECONDS=240 timeout -k 10 900 python3 -u -m pytest tests/test_soak.py -m gpu -k persistent -v -s \
  --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f_soak.txt 2>&1 || { echo "soak failed"; tail -20 gpurun_out/r5f_soak.txt; exit 1; }
grep -E "soak\[|passed|failed" gpurun_out/r5f_soak.txt
