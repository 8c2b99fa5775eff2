#!/bin/bash
# amd-smi concurrency probe + GPU tests + bench.
set -o pipefail
out=gpurun_out/${1:-p3}
mkdir -p $out
timeout -k 10 120 ./build/amdsmi_concurrency > $out/concurrency.txt 2>&1 || { echo "probe failed rc=$?"; cat $out/concurrency.txt; exit 1; }
cat $out/concurrency.txt
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $out/pytest_gpu.txt 2>&1; rc=$?
tail -3 $out/pytest_gpu.txt
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; exit 1; }
timeout -k 10 600 python bench.py --steps 1000 --warmup 100 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; exit 1; }
cat $out/bench.json
