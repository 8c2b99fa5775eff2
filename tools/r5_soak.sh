#!/bin/bash
# A longer soak of the loop daemon on the amd-smi backend (the rewriting writer: leases every cycle):
# RSS, descriptors and gfd-tmp/ must stay flat.  Prints a progress line every 30 s.
set -o pipefail
GFD_SOAK_SECONDS=${1:-300} timeout -k 10 900 python3 -u -m pytest tests/test_soak.py -m gpu -k persistent -v -s \
  --timeout 800 --timeout-method thread -p no:cacheprovider 2>&1 | tee gpurun_out/r5_soak.txt
