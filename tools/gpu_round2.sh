#!/bin/bash
# Soak + write-path probe + rocprofv3 kernel census of one oneshot cycle.
set -o pipefail
out=gpurun_out/${1:-r2}
mkdir -p $out/prof
timeout -k 10 300 python -m pytest tests/test_soak.py -m gpu -q -p no:cacheprovider > $out/soak.txt 2>&1 || { tail -30 $out/soak.txt; exit 1; }
tail -2 $out/soak.txt
timeout -k 5 60 ./build/write_probe $out/wp/gfd > $out/write_probe.txt 2>&1 || exit 1
cat $out/write_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o gfd -- $GRAFT_REPO_ROOT/build/gpu-feature-discovery --oneshot --trace-timing --output-file=$GRAFT_REPO_ROOT/$out/prof/labels > $GRAFT_REPO_ROOT/$out/prof/run.log 2>&1; echo "rocprofv3 rc=$?"
find $GRAFT_REPO_ROOT/$out/prof -type f | head -20
