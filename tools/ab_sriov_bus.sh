#!/bin/bash
# A/B: cycles 1 s apart whose uevent counter moved (tools/uevent_root.py bumps
# it every 0.5 s), the daemon merging the bus's unbound AMD functions on every
# moved counter (GFD_SRIOV_BUS=always) or only inside a VM (unset: on this
# host, the driver listings and the PFs' VF links only).  And the same with the
# counter left alone (the kernel's own), for the steady cost.
set -o pipefail
out=gpurun_out/${1:-ab_sriov_bus}
mkdir -p $out
root=$(mktemp -d /tmp/gfd-uevent-XXXXXX)
python3 tools/uevent_root.py $root --bump 0.5 &
bumper=$!
trap "kill $bumper" EXIT
sleep 1
timeout -k 10 500 python3 tools/cold_cycle.py --backend auto --sysfs-root $root --interval 1s --cycles 20 \
  --variants "GFD_SRIOV_BUS=always,GFD_SRIOV_BUS=vm" --reps 4 --rows > $out/cold.jsonl 2>&1 || exit 1
python3 - $out <<'PY'
import json, statistics, sys
out = sys.argv[1]
per = {}
for line in open(f"{out}/cold.jsonl"):
    if line.startswith('{"variant"'):
        r = json.loads(line)
        per.setdefault(r["variant"], []).append(r)
for v, runs in per.items():
    rows = [row for r in runs for row in r["rows"][1:]]
    moved = [row for row in rows if "pci.bound(checked)" in row or "pci.bound" in row]
    tot = sorted(row["total"] for row in rows)
    med = lambda k, rs: round(statistics.median([x.get(k, 0) for x in rs]), 4) if rs else None
    print(f"{v}: cycles {len(rows)} (counter moved in {len(moved)}) p50 {statistics.median(tot)} p90 {tot[int(0.9*(len(tot)-1))]}"
          f" | run p50s {[r['p50_ms'] for r in runs]} | sriov.self {med('sriov.self', rows)}"
          f" pci.bound(checked) {med('pci.bound(checked)', moved)} pci.list {med('pci.list', moved)} pci.bus {med('pci.bus', moved)}"
          f" pci.vfs {med('pci.vfs', moved)} label {med('label', rows)}")
PY
