#!/usr/bin/env python3
"""A/B of the loop-mode feature-file replace: RENAME_EXCHANGE + deferred unlink
(default) vs rename over the old file (GFD_WRITE_EXCHANGE=never), in the
daemon binary over a synthetic 1-GPU tree, alternated.

    python tools/write_exchange_ab.py [DIR] [--interval 1s] [--cycles 8] [--reps 2]

Output goes to DIR (default /tmp: the file system under test); per run the
cycle, write and replace (write.rename) p50 from --trace-timing, and what
is left in the directory after exit (must be nothing).
"""

from __future__ import annotations

import argparse
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from gpu_feature_discovery_amd.utils import synth  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="/tmp")
    ap.add_argument("--interval", default="1s")
    ap.add_argument("--cycles", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="gfd-xchg-ab-", dir=a.dir)
    fst = subprocess.run(["stat", "-f", "-c", "%T", d], capture_output=True, text=True).stdout.strip()
    root = synth.make_mi355x_node(os.path.join(d, "root"), n_gpus=1)
    print(f"# {d} on {fst}: daemon cycles {a.interval} apart, {a.cycles} per run (first cycle dropped)")
    for rep in range(a.reps):
        for mode in ("never", "default"):
            env = dict(os.environ)
            env.pop("GFD_WRITE_EXCHANGE", None)
            if mode == "never":
                env["GFD_WRITE_EXCHANGE"] = "never"
            out = os.path.join(d, f"out-{mode}-{rep}", "gfd")
            p = subprocess.Popen([os.path.join(REPO, "build", "gpu-feature-discovery"), "--backend=sysfs",
                                  f"--sysfs-root={root}", f"--sleep-interval={a.interval}", "--trace-timing",
                                  f"--output-file={out}", f"--machine-type-file={root}/sys/class/dmi/id/product_name"],
                                 stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=env)
            tot, wr, ren = [], [], []
            for line in p.stderr:
                if "Timing:" not in line:
                    continue
                f = dict(kv.split("=") for kv in line.split("Timing:", 1)[1].split())
                tot.append(float(f["total"][:-2]))
                wr.append(float(f["write"][:-2]))
                ren.append(float(f.get("write.rename", "nanms")[:-2]))
                if len(tot) > a.cycles:
                    break
            p.terminate()
            p.wait(timeout=30)
            left = os.listdir(os.path.dirname(out))
            print(f"rep {rep} GFD_WRITE_EXCHANGE={mode:7s} cycle p50 {statistics.median(tot[1:]):.3f} ms  "
                  f"write p50 {statistics.median(wr[1:]):.3f} ms  replace p50 {statistics.median(ren[1:]):.3f} ms  "
                  f"left after exit: {left}")
    shutil.rmtree(d)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
