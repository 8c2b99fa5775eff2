#!/usr/bin/env python3
"""What a sleeping daemon holds on the GPU (verdict r5, Next #1).

Starts the daemon loop under each backend with a long sleep interval, waits
until the amd-smi session (if any) is in use and the daemon logged
"Sleeping for", then records:

* every descriptor (`readlink /proc/<pid>/fd/*`), marking /dev/kfd and
  /dev/dri/* ones;
* whether KFD lists the process (`/sys/class/kfd/kfd/proc/<pid>`);
* the process's memory maps of /dev/kfd or /dev/dri (`/proc/<pid>/maps`).

Usage: tools/hold_probe.py [--binary PATH] [--sleep 5s] [backend ...]
Prints one JSON object per backend.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from gpu_feature_discovery_amd.utils.proc import gpu_holds  # noqa: E402


def probe(binary: str, backend: str, sleep: str, out_dir: Path, wait_for: str, timeout: float = 60) -> dict:
    out = out_dir / f"gfd-{backend}"
    env = {k: v for k, v in os.environ.items() if not k.startswith("GFD_")}
    p = subprocess.Popen([binary, f"--sleep-interval={sleep}", f"--backend={backend}", f"--output-file={out}"],
                         env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    err, seen, res = [], not wait_for, {}
    try:
        deadline = time.monotonic() + timeout
        for line in p.stderr:
            err.append(line)
            seen = seen or wait_for in line
            if seen and "Sleeping for" in line:
                time.sleep(0.3)  # well inside the sleep
                res = gpu_holds(p.pid)
                break
            if time.monotonic() > deadline:
                break
    finally:
        p.send_signal(signal.SIGTERM)
        _, rest = p.communicate(timeout=30)
        err.append(rest or "")
    res.update({"backend": backend, "sleep": sleep, "rc": p.returncode, "log_tail": "".join(err)[-1500:]})
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--binary", default=str(REPO / "build" / "gpu-feature-discovery"))
    ap.add_argument("--sleep", default="5s")
    ap.add_argument("--out", default="/tmp/hold_probe")
    ap.add_argument("backends", nargs="*", default=["auto", "amdsmi", "sysfs"])
    a = ap.parse_args()
    out_dir = Path(a.out)
    out_dir.mkdir(parents=True, exist_ok=True)
    waits = {"auto": "Using the amdsmi", "amdsmi": "", "sysfs": ""}
    for b in a.backends:
        print(json.dumps(probe(a.binary, b, a.sleep, out_dir, waits.get(b, ""))), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
