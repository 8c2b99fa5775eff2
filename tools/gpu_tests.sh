#!/bin/bash
# GPU test pass: pytest -m gpu, then the bench.
set -o pipefail
out=gpurun_out/${1:-t1}
mkdir -p $out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $out/pytest_gpu.txt 2>&1; rc=$?
tail -5 $out/pytest_gpu.txt
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; exit 1; }
timeout -k 10 600 python bench.py --steps 500 --warmup 50 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; exit 1; }
cat $out/bench.json
