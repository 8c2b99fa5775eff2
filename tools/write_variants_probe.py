#!/usr/bin/env python3
"""Per-variant cost of replacing a small file atomically in DIR (default: a
new directory under /tmp), median of N: the daemon's way (create a named
temp file in DIR/gfd-tmp, write, close, rename over DIR/out) vs an unnamed
O_TMPFILE linked into gfd-tmp (linkat through /proc/self/fd) then renamed.
Both keep the reference's semantics (every cycle a new inode, renamed over
the old one); the question is only which is cheaper on the file system.

    python tools/write_variants_probe.py [DIR] [N]
"""

from __future__ import annotations

import ctypes
import os
import statistics
import sys
import tempfile
import time

data = b"x" * 1200  # about one node's label file
_libc = ctypes.CDLL(None, use_errno=True)
_AT_FDCWD, _AT_SYMLINK_FOLLOW = -100, 0x400


def _linkat_follow(src: str, dst: str) -> None:
    # os.link() calls link(2), which does not dereference /proc/self/fd/N.
    if _libc.linkat(_AT_FDCWD, src.encode(), _AT_FDCWD, dst.encode(), _AT_SYMLINK_FOLLOW) != 0:
        e = ctypes.get_errno()
        raise OSError(e, os.strerror(e))


def named(d: str, i: int) -> None:
    p = os.path.join(d, "gfd-tmp", f"gfd-{i}")
    fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_EXCL | os.O_CLOEXEC, 0o644)
    os.write(fd, data)
    os.close(fd)
    os.rename(p, os.path.join(d, "out"))


def tmpfile(d: str, i: int) -> None:
    fd = os.open(os.path.join(d, "gfd-tmp"), os.O_WRONLY | os.O_TMPFILE | os.O_CLOEXEC, 0o644)
    os.write(fd, data)
    p = os.path.join(d, "gfd-tmp", f"gfd-{i}")
    _linkat_follow(f"/proc/self/fd/{fd}", p)
    os.close(fd)
    os.rename(p, os.path.join(d, "out"))


def main() -> int:
    base = sys.argv[1] if len(sys.argv) > 1 else None
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    d = tempfile.mkdtemp(prefix="gfd-wv-", dir=base)
    os.makedirs(os.path.join(d, "gfd-tmp"))
    print(f"directory {d}")
    for rep in range(3):
        for name, fn in (("named temp + rename", named), ("O_TMPFILE + linkat + rename", tmpfile)):
            xs = []
            try:
                for i in range(n):
                    t0 = time.perf_counter_ns()
                    fn(d, rep * 10 * n + i + (0 if fn is named else 5 * n))
                    xs.append((time.perf_counter_ns() - t0) / 1e3)
            except OSError as e:
                print(f"  {name}: {e}")
                continue
            print(f"  rep {rep} {name:30s} p50 {statistics.median(xs):7.2f} us  p90 {sorted(xs)[int(0.9 * n)]:7.2f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
