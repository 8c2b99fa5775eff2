#!/bin/bash
# A longer soak of the loop daemon on the amd-smi backend (the rewriting writer: leases every cycle, a
# reader of the feature file running throughout): RSS, descriptors and gfd-tmp/ must stay flat.  Prints a
# progress line every 30 s.  Usage (GPU box): tools/soak.sh [seconds, default 300]
set -o pipefail
s=${1:-300}
GFD_SOAK_SECONDS=$s timeout -k 10 $((s + 240)) python3 -u -m pytest tests/test_soak.py -m gpu -k persistent -v -s \
  --timeout $((s + 180)) --timeout-method thread -p no:cacheprovider 2>&1 | tee gpurun_out/soak.txt
