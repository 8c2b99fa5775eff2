#!/usr/bin/env python3
"""RSS / descriptor series of the daemon in a tight loop (1 ms interval),
sampled every --every seconds for --seconds: a leak grows linearly with
cycles, allocator warm-up plateaus.

    python tools/rss_series.py [--seconds 300] [--every 20] [--backend amdsmi]
        [--backend sysfs --sysfs-root synthetic|PATH]
"""

from __future__ import annotations

import argparse
import os
import signal
import subprocess
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mem_kib(pid: int) -> dict[str, int]:
    """VmRSS and its split: RssAnon (heap, stacks: what a leak grows) and
    RssFile (mapped code and data touched so far: grows as rarely taken paths
    of the binary and its libraries run for the first time, then stops)."""
    out = {}
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            k = line.split(":")[0]
            if k in ("VmRSS", "RssAnon", "RssFile", "Threads"):
                out[k] = int(line.split()[1])
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--every", type=float, default=20)
    ap.add_argument("--backend", default="amdsmi")
    ap.add_argument("--sysfs-root", default=None, help="a synthetic node (utils/synth.py) instead of the host")
    ap.add_argument("--arg", action="append", default=[], help="extra daemon argument (repeatable)")
    ap.add_argument("--binary", default=os.path.join(REPO, "build", "gpu-feature-discovery"),
                    help="daemon binary (e.g. an older build staged for an A/B)")
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="gfd-rss-")
    out = os.path.join(d, "gfd")
    extra = []
    if a.sysfs_root == "synthetic":
        import sys

        sys.path.insert(0, REPO)
        from gpu_feature_discovery_amd.utils import synth

        a.sysfs_root = str(synth.make_mi355x_node(os.path.join(d, "node"), n_gpus=8, seed=3))
    if a.sysfs_root:
        extra = [f"--sysfs-root={a.sysfs_root}", f"--machine-type-file={a.sysfs_root}/sys/class/dmi/id/product_name"]
    p = subprocess.Popen([a.binary, f"--backend={a.backend}", *extra,
                          "--sleep-interval=1ms", "--trace-timing", f"--output-file={out}", *a.arg],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    cycles = [0]
    # Cycles that did more than the steady state, by what the Timing line
    # names: an amd-smi re-initialisation (the KFD topology generation moved:
    # another GPU of the host reset or re-partitioned), an SR-IOV check after
    # an unrelated uevent, an SR-IOV re-read.
    events = {"amdsmi_init=": 0, "pci.bound(checked)=": 0, "pci.drivers=": 0}

    def reader():
        for line in p.stderr:
            if "Timing:" in line:
                cycles[0] += 1
                for k in events:
                    if k in line:
                        events[k] += 1

    threading.Thread(target=reader, daemon=True).start()
    t0 = time.monotonic()
    try:
        while time.monotonic() - t0 < a.seconds and p.poll() is None:
            time.sleep(a.every)
            m = mem_kib(p.pid)
            print(f"t={time.monotonic() - t0:6.0f}s cycles={cycles[0]:8d} rss={m.get('VmRSS')} KiB "
                  f"(anon {m.get('RssAnon')}, file {m.get('RssFile')}) fds={len(os.listdir(f'/proc/{p.pid}/fd'))} "
                  f"threads={m.get('Threads')} "
                  f"reinit={events['amdsmi_init=']} sriov_checked={events['pci.bound(checked)=']} "
                  f"sriov_reread={events['pci.drivers=']}",
                  flush=True)
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=30)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
