#!/bin/bash
# One GPU pass (what each round records under profiles/): the GPU test suite,
# the benchmark as the driver runs it, and the oneshot (Job-mode) breakdown.
# Every step is time-limited and the first failure ends the pass.
# Usage (GPU box): tools/gpu_pass.sh [outdir-name] [bench args...]
set -o pipefail
out=gpurun_out/${1:-gpu_pass}
shift || true
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$out/pytest_gpu.txt" 2>&1; rc=$?
tail -3 "$out/pytest_gpu.txt"
[ $rc -eq 0 ] || { echo "pytest -m gpu failed rc=$rc"; exit 1; }
timeout -k 10 400 python bench.py "$@" > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; exit 1; }
tail -c 400 "$out/bench.json"
timeout -k 10 300 tools/oneshot_breakdown.sh "$(basename "$out")/breakdown" > /dev/null || { echo "breakdown failed"; exit 1; }
echo "pass ok: $out"
