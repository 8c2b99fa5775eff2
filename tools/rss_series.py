#!/usr/bin/env python3
"""RSS / descriptor series of the daemon in a tight loop (1 ms interval),
sampled every --every seconds for --seconds: a leak grows linearly with
cycles, allocator warm-up plateaus.

    python tools/rss_series.py [--seconds 300] [--every 20] [--backend amdsmi]
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


def rss_kib(pid: int) -> int:
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--every", type=float, default=20)
    ap.add_argument("--backend", default="amdsmi")
    a = ap.parse_args()
    out = os.path.join(tempfile.mkdtemp(prefix="gfd-rss-"), "gfd")
    p = subprocess.Popen([os.path.join(REPO, "build", "gpu-feature-discovery"), f"--backend={a.backend}",
                          "--sleep-interval=1ms", "--trace-timing", f"--output-file={out}"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    cycles = [0]

    def reader():
        for line in p.stderr:
            if "Timing:" in line:
                cycles[0] += 1

    threading.Thread(target=reader, daemon=True).start()
    t0 = time.monotonic()
    try:
        while time.monotonic() - t0 < a.seconds and p.poll() is None:
            time.sleep(a.every)
            print(f"t={time.monotonic() - t0:6.0f}s cycles={cycles[0]:8d} rss={rss_kib(p.pid)} KiB "
                  f"fds={len(os.listdir(f'/proc/{p.pid}/fd'))}", flush=True)
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=30)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
