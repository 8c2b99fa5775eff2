#!/usr/bin/env python3
"""Cycle latency of the daemon as deployed: a real sleep between cycles
(cores idle, workers parked, caches cold), read from its own --trace-timing.

    python tools/cold_cycle.py [--interval 2s] [--cycles 40] [--backend amdsmi]
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import statistics
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--interval", default="2s")
    ap.add_argument("--cycles", type=int, default=40)
    ap.add_argument("--backend", default="amdsmi")
    ap.add_argument("--sysfs-root", default=None)
    ap.add_argument("--visible-devices", default="")
    a = ap.parse_args()
    extra = [f"--visible-devices={a.visible_devices}"]
    if a.sysfs_root:
        extra += [f"--sysfs-root={a.sysfs_root}", f"--machine-type-file={a.sysfs_root}/sys/class/dmi/id/product_name"]
    out = os.path.join(tempfile.mkdtemp(prefix="gfd-cold-"), "gfd")
    p = subprocess.Popen([os.path.join(REPO, "build", "gpu-feature-discovery"), f"--backend={a.backend}",
                          f"--sleep-interval={a.interval}", "--trace-timing", f"--output-file={out}", *extra],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    totals, phases = [], {}
    try:
        for line in p.stderr:
            if "Timing:" not in line:
                continue
            fields = dict(kv.split("=") for kv in line.split("Timing:", 1)[1].split())
            totals.append(float(fields["total"].rstrip("ms")))
            if len(totals) > 1:
                for k, v in fields.items():
                    phases.setdefault(k, []).append(float(v.rstrip("ms")))
            print(f"cycle {len(totals)}: {fields['total']}", file=sys.stderr, flush=True)
            if len(totals) >= a.cycles:
                break
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=30)
    steady = totals[1:]
    print(json.dumps({"interval": a.interval, "backend": a.backend, "cycles": len(totals),
                      "first_cycle_ms": totals[0], "p50_ms": round(statistics.median(steady), 4),
                      "p90_ms": round(sorted(steady)[int(0.9 * (len(steady) - 1))], 4),
                      "phases_p50_ms": {k: round(statistics.median(v), 4) for k, v in phases.items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
