#!/bin/bash
# A/B of one environment setting on Job processes (--oneshot, null and auto
# backends), alternated: the default vs VAR=value, spawn to exit with a
# blocking waitpid, 30 processes per point; then one --trace-timing cycle
# per mode (where the SR-IOV scan's time goes).
# Usage (GPU box): tools/oneshot_env_ab.sh <outdir-name> <reps> VAR=value
set -o pipefail
out=gpurun_out/${1:?outdir}
mkdir -p "$out"
python3 - "$out" "${2:?reps}" "${3:?VAR=value}" <<'PY' | tee "$out/ab.txt"
import os, statistics, subprocess, sys
sys.path.insert(0, ".")
from gpu_feature_discovery_amd.utils.proc import spawn_wait_ms
out, reps, setting = sys.argv[1], int(sys.argv[2]), sys.argv[3]
var, val = setting.split("=", 1)
binary = "./build/gpu-feature-discovery"
def env_for(mode):
    env = {k: v for k, v in os.environ.items() if k != var}
    if mode != "default":
        env[var] = val
    return env
for r in range(reps):
    for mode in ("default", setting):
        for backend in ("null", "auto"):
            xs = sorted(spawn_wait_ms([binary, "--oneshot", f"--backend={backend}", f"--output-file={out}/gfd"],
                                      timeout=60, env=env_for(mode)) for _ in range(30))
            print(f"rep {r} {mode:24s} oneshot {backend:4s}: p50 {statistics.median(xs):.3f} ms  p90 {xs[27]:.3f} ms")
for mode in ("default", setting):
    for _ in range(3):
        cp = subprocess.run([binary, "--oneshot", "--backend=null", "--trace-timing", f"--output-file={out}/gfd"],
                            capture_output=True, text=True, timeout=60, env=env_for(mode))
        print(f"{mode:24s} " + " ".join(l.split("Timing:", 1)[1].strip() for l in cp.stderr.splitlines() if " Timing:" in l))
PY
