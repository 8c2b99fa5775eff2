#!/usr/bin/env python3
"""A/B of feature-file write modes in the daemon binary at the deployed
cadence: loop mode with a real sleep between cycles, each variant an
environment setting, alternated; per run the cycle, write and replace p50
from --trace-timing, and what is left in the output directory after exit.

    python tools/writer_ab.py [DIR] [--interval 1s] [--cycles 10] [--reps 3]
        [--backend auto|synthetic] [--variant VAR=val[,VAR=val]] ...

DIR is where the output file goes (its file system is what is measured).
A variant's BIN=path runs that daemon binary instead of build/'s (e.g. an
earlier commit's build, to compare revisions on one box).
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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="/tmp")
    ap.add_argument("--interval", default="1s")
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--variant", action="append", default=[])
    a = ap.parse_args()
    variants = ["default"] + a.variant
    d = tempfile.mkdtemp(prefix="gfd-writer-ab-", dir=a.dir)
    fst = subprocess.run(["stat", "-f", "-c", "%T", d], capture_output=True, text=True).stdout.strip()
    extra = [f"--backend={a.backend}"]
    if a.backend == "synthetic":
        from gpu_feature_discovery_amd.utils import synth

        root = synth.make_mi355x_node(os.path.join(d, "root"), n_gpus=1)
        extra = ["--backend=sysfs", f"--sysfs-root={root}", f"--machine-type-file={root}/sys/class/dmi/id/product_name"]
    print(f"# {d} on {fst}: {a.backend} backend, daemon cycles {a.interval} apart, {a.cycles} per run "
          f"(first cycle dropped)", flush=True)
    for rep in range(a.reps):
        for i, var in enumerate(variants):
            env = dict(os.environ)
            for v in variants[1:]:
                for kv in v.split(","):
                    env.pop(kv.split("=", 1)[0], None)
            binary = os.path.join(REPO, "build", "gpu-feature-discovery")
            if var != "default":
                env.update(kv.split("=", 1) for kv in var.split(","))
                binary = os.path.join(REPO, env.pop("BIN", binary))
            out = os.path.join(d, f"out-{i}-{rep}", "gfd")
            p = subprocess.Popen([binary, *extra,
                                  f"--sleep-interval={a.interval}", "--trace-timing", f"--output-file={out}"],
                                 stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=env)
            tot, wr, ren = [], [], []
            for line in p.stderr:
                if "Timing:" not in line:
                    continue
                f = dict(kv.split("=") for kv in line.split("Timing:", 1)[1].split())
                tot.append(float(f["total"][:-2]))
                wr.append(float(f.get("write", "nanms")[:-2]))
                ren.append(float(f.get("write.rename", "nanms")[:-2]))
                if len(tot) > a.cycles:
                    break
            p.terminate()
            p.wait(timeout=30)
            left = sorted(os.listdir(os.path.dirname(out)))
            print(f"rep {rep} {var:60s} cycle p50 {statistics.median(tot[1:]):.3f} ms  "
                  f"write p50 {statistics.median(wr[1:]):.3f} ms  replace p50 {statistics.median(ren[1:]):.3f} ms "
                  f"max {max(ren[1:]):.3f} ms  "
                  f"left after exit: {left}", flush=True)
    shutil.rmtree(d)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
