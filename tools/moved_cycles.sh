#!/bin/bash
# Cycles 1 s apart in which the uevent counter moved (tools/uevent_root.py
# bumps it every 0.5 s) - the cost of the SR-IOV re-check - next to cycles
# with the kernel's own counter (mostly unmoved), alternated.
set -o pipefail
out=gpurun_out/${1:-moved_cycles}
mkdir -p $out
root=$(mktemp -d /tmp/gfd-uevent-XXXXXX)
python3 tools/uevent_root.py $root --bump 0.5 &
bumper=$!
trap "kill $bumper" EXIT
sleep 1
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/cold_cycle.py --backend auto --sysfs-root $root --interval 1s --cycles 20 --rows \
    > $out/moved_$rep.jsonl 2>&1 || exit 1
  timeout -k 10 120 python3 tools/cold_cycle.py --backend auto --interval 1s --cycles 20 --rows \
    > $out/real_$rep.jsonl 2>&1 || exit 1
done
python3 - $out <<'PY'
import json, statistics, sys, glob
out = sys.argv[1]
for kind in ("moved", "real"):
    runs = [json.loads(l) for f in sorted(glob.glob(f"{out}/{kind}_*.jsonl")) for l in open(f) if l.startswith('{"variant"')]
    rows = [row for r in runs for row in r["rows"][1:]]
    moved = [row for row in rows if "pci.bound(checked)" in row or "pci.bound" in row]
    tot = sorted(row["total"] for row in rows)
    med = lambda k, rs: round(statistics.median([x.get(k, 0) for x in rs]), 4) if rs else None
    print(f"{kind}: cycles {len(rows)} (counter moved in {len(moved)}) p50 {statistics.median(tot)} p90 {tot[int(0.9*(len(tot)-1))]}"
          f" | run p50s {[r['p50_ms'] for r in runs]} | moved cycles: total {med('total', moved)} pci.bound(checked) "
          f"{med('pci.bound(checked)', moved)} pci.list {med('pci.list', moved)} pci.vfs {med('pci.vfs', moved)}")
PY
