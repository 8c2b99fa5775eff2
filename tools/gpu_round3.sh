#!/bin/bash
# GPU pass: pytest -m gpu, the bench, in-process per-call amd-smi trace and
# the PCI scan probe.  Every step is time-limited; the first failure ends it.
set -o pipefail
out=gpurun_out/${1:-r3}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $out/pytest_gpu.txt 2>&1; rc=$?
tail -5 $out/pytest_gpu.txt
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; exit 1; }
timeout -k 10 600 python bench.py --steps 1000 --warmup 100 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; exit 1; }
cat $out/bench.json
timeout -k 10 300 python tools/inproc_trace.py 500 > $out/inproc_trace.txt 2>&1 || { echo "inproc trace failed"; exit 1; }
cat $out/inproc_trace.txt
timeout -k 5 60 ./build/pci_scan_probe > $out/pci_scan_probe.txt 2>&1 || { echo "pci probe failed"; exit 1; }
cat $out/pci_scan_probe.txt
