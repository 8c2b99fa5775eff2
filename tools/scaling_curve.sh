#!/bin/bash
# 1/2/4/8-GPU curves that a one-GPU box can produce: the KFD-sysfs backend
# over synthetic MI355X trees (bench.py --backend synthetic, one process),
# and the amd-smi backend over the latency-modelled fake library.
set -o pipefail
out=gpurun_out/${1:-scaling}
mkdir -p $out
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --gpus $n --steps 1000 --warmup 100 --backend synthetic --no-extras \
    > $out/synthetic_$n.json 2> $out/synthetic_$n.err || exit 1
done
timeout -k 10 300 python tools/fake_scaling.py --steps 1000 > $out/fake_scaling.json 2> $out/fake_scaling.err || exit 1
python3 - "$out" <<'PY'
import json, sys
out = sys.argv[1]
rows = []
for n in (1, 2, 4, 8):
    r = json.loads(open(f"{out}/synthetic_{n}.json").read().strip().splitlines()[-1])
    rows.append({"gpus": n, "p50_ms": r["value"], "p90_ms": r["p90_ms"], "labels_ok": r["labels_ok"]})
fake = json.load(open(f"{out}/fake_scaling.json"))
json.dump({"sysfs_backend_synthetic_tree": rows, "amdsmi_backend_fake_library": fake}, open(f"{out}/curve.json", "w"),
          indent=1)
print(open(f"{out}/curve.json").read())
PY
