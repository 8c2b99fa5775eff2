#!/bin/bash
# rocprofv3 kernel and memory-copy traces of one oneshot labeling run per
# backend (GPU box): the daemon dispatches no kernels and copies nothing, so
# rocprofv3 writes no trace or stats files; the log and the file listing say
# so.  Output: gpurun_out/${1:-rocprof}/{log_amdsmi,log_auto}.txt.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-rocprof}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
for b in amdsmi auto; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/$b -o run -- $R/build/gpu-feature-discovery --oneshot --backend=$b --trace-timing --output-file=$O/labels_$b > $O/log_$b.txt 2>&1 || { echo "rocprof $b failed rc=$?"; exit 1; }
  echo "== files written under $O/$b:" >> $O/log_$b.txt; (find $O/$b -type f 2>/dev/null || true) >> $O/log_$b.txt
done
echo done
