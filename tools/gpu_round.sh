#!/bin/bash
# One GPU verification pass: smoke, daemon oneshot on both backends, bench.
set -o pipefail
out=gpurun_out/${1:-r1}
mkdir -p $out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { echo "smoke failed rc=$?"; exit 1; }
timeout -k 10 60 ./build/gpu-feature-discovery --oneshot -o $out/gfd-amdsmi --trace-timing > $out/daemon-amdsmi.log 2>&1 || { echo "daemon amdsmi failed"; exit 1; }
timeout -k 10 60 ./build/gpu-feature-discovery --oneshot -o $out/gfd-sysfs --backend=sysfs --trace-timing > $out/daemon-sysfs.log 2>&1 || { echo "daemon sysfs failed"; exit 1; }
timeout -k 10 600 python bench.py --steps 200 --warmup 20 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; exit 1; }
cat $out/bench.json
