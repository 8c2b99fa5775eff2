#!/bin/bash
# How the daemon's backends react to environment variables a GPU pod may
# carry (device-plugin / runtime visibility masks).  Each run: oneshot,
# labels to stdout, the gpu.count label and the backend line.
# Usage (GPU box): tools/env_probe.sh > gpurun_out/env_probe.txt
bin=build/gpu-feature-discovery
for backend in amdsmi sysfs auto; do
  for env in "" "ROCR_VISIBLE_DEVICES=1" "HIP_VISIBLE_DEVICES=1" "CUDA_VISIBLE_DEVICES=1" "GPU_DEVICE_ORDINAL=1" \
             "ROCR_VISIBLE_DEVICES=0" "HSA_ENABLE_IPC_MODE_LEGACY=1"; do
    out=$(env $env timeout -k 5 60 $bin --oneshot --no-timestamp --backend=$backend --output-file= 2>/tmp/err.txt)
    rc=$?
    echo "backend=$backend env='${env}' rc=$rc count=$(echo "$out" | sed -n 's/^amd.com\/gpu.count=//p') \
product=$(echo "$out" | sed -n 's/^amd.com\/gpu.product=//p') $(grep -o 'Using [^ ]* manager' /tmp/err.txt | head -1)"
  done
done
