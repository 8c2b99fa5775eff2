#!/usr/bin/env python3
"""Cold feature-file replace: rename over the old file vs exchange + deferred unlink.

    python tools/rename_exchange_probe.py [DIR] [--cycles 12] [--interval 1.0]

Each cycle (DIR idle for --interval seconds before it, as in the deployed
daemon) writes a preallocated 2 KB temp file in DIR/gfd-tmp and then either
  rename   - rename(tmp, out): the old file's inode is dropped inside the call
  exchange - renameat2(tmp, out, RENAME_EXCHANGE): the two names swap
             atomically, and the old contents (now under the temp name) are
             unlinked afterwards, timed apart (the daemon would do it on a worker)
Modes alternate cycle by cycle; medians of the replace call are printed.
"""

from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import subprocess
import tempfile
import time

AT_FDCWD = -100
RENAME_EXCHANGE = 2
SYS_renameat2 = 316  # x86-64

libc = ctypes.CDLL(None, use_errno=True)


def renameat2(a: str, b: str, flags: int) -> None:
    r = libc.syscall(SYS_renameat2, AT_FDCWD, a.encode(), AT_FDCWD, b.encode(), flags)
    if r != 0:
        e = ctypes.get_errno()
        raise OSError(e, os.strerror(e))


def make_tmp(d: str, i: int, data: bytes) -> str:
    p = os.path.join(d, f"gfd-{i:06d}")
    fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o644)
    os.posix_fallocate(fd, 0, len(data))
    os.write(fd, data)
    os.close(fd)
    return p


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?")
    ap.add_argument("--cycles", type=int, default=12)
    ap.add_argument("--interval", type=float, default=1.0)
    a = ap.parse_args()
    base = tempfile.mkdtemp(prefix="gfd-xchg-", dir=a.dir)
    fst = subprocess.run(["stat", "-f", "-c", "%T", base], capture_output=True, text=True).stdout.strip()
    tmpd = os.path.join(base, "gfd-tmp")
    os.mkdir(tmpd)
    out = os.path.join(base, "gfd")
    data = b"".join(b"amd.com/label-%02d=value-%040d\n" % (k, k) for k in range(32))
    make_tmp(tmpd, 0, data)
    os.rename(os.path.join(tmpd, "gfd-000000"), out)
    res: dict[str, list[float]] = {"rename": [], "exchange": [], "exchange.unlink": []}
    for i in range(1, 2 * a.cycles + 1):
        time.sleep(a.interval)
        p = make_tmp(tmpd, i, data)
        mode = "rename" if i % 2 else "exchange"
        t0 = time.perf_counter_ns()
        if mode == "rename":
            os.rename(p, out)
            res[mode].append((time.perf_counter_ns() - t0) / 1e6)
        else:
            renameat2(p, out, RENAME_EXCHANGE)
            t1 = time.perf_counter_ns()
            os.unlink(p)  # the old contents, now under the temp name
            t2 = time.perf_counter_ns()
            res[mode].append((t1 - t0) / 1e6)
            res["exchange.unlink"].append((t2 - t1) / 1e6)
    print(f"# {base} on {fst}, {a.cycles} cycles per mode, {a.interval:g} s apart, 2 KB preallocated file")
    for k, xs in res.items():
        xs.sort()
        print(f"{k:16s} p50 {statistics.median(xs):.4f} ms  p90 {xs[int(0.9 * (len(xs) - 1))]:.4f} ms  max {xs[-1]:.4f} ms")
    for f in os.listdir(tmpd):
        os.unlink(os.path.join(tmpd, f))
    os.rmdir(tmpd)
    os.unlink(out)
    os.rmdir(base)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
