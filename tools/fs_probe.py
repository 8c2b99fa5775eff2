#!/usr/bin/env python3
"""Latency of the feature-file write's file-system operations, per
directory: the daemon's atomic replace (create in gfd-tmp/, write, close,
rename into the output directory) and its variants (same-directory rename,
RENAME_EXCHANGE), plus the file system type and the host's dirty pages.

    python tools/fs_probe.py [--iters 200] [DIR ...]

Run as the first command of a fresh box, then again later, to see whether
a fresh box's slow writes are its file system settling and which directory
(/tmp, /dev/shm, the repository) they hit.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import tempfile
import time

RENAME_EXCHANGE = 2
libc = ctypes.CDLL(None, use_errno=True)
FS_NAMES = {0xEF53: "ext4", 0x794C7630: "overlay", 0x01021994: "tmpfs", 0x58465342: "xfs", 0x9123683E: "btrfs"}


def fstype(path: str) -> str:
    class Statfs(ctypes.Structure):
        _fields_ = [("f_type", ctypes.c_long), ("rest", ctypes.c_char * 112)]

    s = Statfs()
    if libc.statfs(path.encode(), ctypes.byref(s)) != 0:
        return "?"
    return FS_NAMES.get(s.f_type & 0xFFFFFFFF, hex(s.f_type & 0xFFFFFFFF))


def renameat2(a: str, b: str, flags: int) -> None:
    if libc.renameat2(-100, a.encode(), -100, b.encode(), flags) != 0:
        raise OSError(ctypes.get_errno(), os.strerror(ctypes.get_errno()))


def probe(base: str, iters: int) -> dict:
    d = tempfile.mkdtemp(prefix="gfd-fsprobe-", dir=base)
    tmp = os.path.join(d, "gfd-tmp")
    os.mkdir(tmp)
    out = os.path.join(d, "gfd")
    data = b"amd.com/gpu.count=1\n" * 40
    ops: dict[str, list[float]] = {}

    def t(name, fn, *args):
        t0 = time.perf_counter_ns()
        r = fn(*args)
        ops.setdefault(name, []).append((time.perf_counter_ns() - t0) / 1e3)
        return r

    for i in range(iters):
        name = os.path.join(tmp, f"gfd-amd-{i:06d}")
        fd = t("create", os.open, name, os.O_WRONLY | os.O_CREAT | os.O_EXCL | os.O_CLOEXEC, 0o644)
        t("write", os.write, fd, data)
        t("close", os.close, fd)
        if i % 3 == 0:
            t("rename_xdir", os.rename, name, out)
        elif i % 3 == 1 and os.path.exists(out):
            t("exchange", renameat2, name, out, RENAME_EXCHANGE)
            t("unlink", os.unlink, name)
        else:
            same = os.path.join(d, f".gfd-amd-{i:06d}")
            os.rename(name, same)
            t("rename_samedir", os.rename, same, out)
    for f in os.listdir(tmp):
        os.unlink(os.path.join(tmp, f))
    os.rmdir(tmp)
    os.unlink(out)
    os.rmdir(d)
    return {"dir": base, "fs": fstype(base), **{k: round(statistics.median(v), 2) for k, v in ops.items()},
            "p90": {k: round(sorted(v)[int(len(v) * 0.9)], 2) for k, v in ops.items()}}


def dirty() -> str:
    with open("/proc/meminfo") as f:
        return " ".join(ln.split(":")[0] + "=" + ln.split()[1] for ln in f if ln.startswith(("Dirty", "Writeback:")))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("dirs", nargs="*")
    a = ap.parse_args()
    dirs = a.dirs or [tempfile.gettempdir(), "/dev/shm", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
    print(json.dumps({"t": round(time.monotonic(), 1), "meminfo_kB": dirty()}), flush=True)
    for base in dirs:
        if os.path.isdir(base) and os.access(base, os.W_OK):
            print(json.dumps({"us_median": probe(base, a.iters)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
