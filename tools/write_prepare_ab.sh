#!/bin/bash
# A/B of the prepared temporary file (src/lm/labels.cpp, prepare_next): the
# bench with GFD_WRITE_PREPARE=never (every write creates its file) vs the
# default (a worker creates the next cycle's file after each rename),
# alternated on one box.  Also times /proc/bus/pci/devices read in page-sized
# vs large chunks (the cold SR-IOV scan's device table, util/fs.cpp).
# Usage (GPU box): tools/write_prepare_ab.sh [outdir-name] [reps]
set -o pipefail
out=gpurun_out/${1:-write_prepare_ab}
reps=${2:-2}
mkdir -p "$out"
python3 - <<'PY' | tee "$out/proc_table.txt"
import os, time
def rd(bs):
    fd = os.open("/proc/bus/pci/devices", os.O_RDONLY)
    n, calls = 0, 0
    while True:
        b = os.read(fd, bs)
        calls += 1
        if not b:
            break
        n += len(b)
    os.close(fd)
    return n, calls
for bs in (4096, 65536, 1 << 20):
    ts = []
    for _ in range(200):
        t = time.perf_counter_ns(); n, calls = rd(bs); ts.append(time.perf_counter_ns() - t)
    ts.sort()
    print(f"/proc/bus/pci/devices ({n} bytes) read in {bs:7d}-byte chunks ({calls} reads): p50 {ts[100]/1e3:7.1f} us  p90 {ts[180]/1e3:7.1f} us")
PY
for r in $(seq 1 $reps); do
  for mode in never default; do
    if [ $mode = never ]; then export GFD_WRITE_PREPARE=never; else unset GFD_WRITE_PREPARE; fi
    timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $out/${mode}_$r.json 2> $out/${mode}_$r.err \
      || { echo "bench failed"; tail -5 $out/${mode}_$r.err; exit 1; }
    python3 -c "
import json; r = json.load(open('$out/${mode}_$r.json')); e = r['extras']; c = r['cold_cycle'] or {}
print('rep $r %-7s: hot p50 %.4f p90 %.4f (write %.4f) ms/step %.4f | daemon loop p50 %.4f | cold p50 %.3f (write %.3f) | first %.3f | Job %.3f' % (
  '$mode', r['value'], r['p90_ms'], r['phases_p50_ms'].get('write', 0), r['ms_per_step'], e['daemon_loop']['p50_ms'],
  c.get('p50_ms', 0), c.get('phases_p50_ms', {}).get('write', 0), r['first_cycle_ms'] or 0, r['oneshot_process_p50_ms'] or 0))"
  done
done | tee $out/ab.txt
