#!/usr/bin/env python3
"""A/B of the feature-file write on the file system of a directory.

    python tools/write_ext4_ab.py [DIR]      (default: a temp dir under /tmp)

Part 1 - syscall level: create a temp file in DIR/gfd-tmp, write ~2 KB (the
size of a node's label file), close, rename over DIR/out; per-syscall medians
with and without fallocate(2) before the write, and with the target unlinked
first (no replace).  On ext4 (auto_da_alloc) the replacing rename flushes the
new file's delayed-allocation blocks; preallocating leaves none.

Part 2 - the daemon's writer (bench.py over the synthetic tree, output in
DIR): GFD_WRITE_PREALLOC=never vs the default (auto: ext4/overlayfs).
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fs_type(path: str) -> str:
    out = subprocess.run(["stat", "-f", "-c", "%T", path], capture_output=True, text=True)
    return out.stdout.strip() or "?"


def syscall_ab(d: str, n: int = 30) -> None:
    import time

    os.makedirs(os.path.join(d, "gfd-tmp"), exist_ok=True)
    data = b"x" * 2000
    out = os.path.join(d, "out")
    for mode in ("plain", "unlink_first", "fallocate", "plain", "fallocate"):
        ts: dict[str, list[float]] = {}
        for i in range(n):
            p = os.path.join(d, "gfd-tmp", f"a{i}")
            t0 = time.perf_counter()
            fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o644)
            t1 = time.perf_counter()
            if mode == "fallocate":
                os.posix_fallocate(fd, 0, len(data))
            os.write(fd, data)
            os.close(fd)
            t2 = time.perf_counter()
            if mode == "unlink_first" and os.path.exists(out):
                os.unlink(out)
            os.rename(p, out)
            t3 = time.perf_counter()
            for k, v in (("open", t1 - t0), ("write+close", t2 - t1), ("rename", t3 - t2)):
                ts.setdefault(k, []).append(v * 1e3)
        med = {k: round(sorted(v)[n // 2], 3) for k, v in ts.items()}
        mx = {k: round(max(v), 3) for k, v in ts.items()}
        print(f"  {mode:13s} median ms {med}  max ms {mx}")


def bench_ab(d: str) -> None:
    for mode in ("never", "auto"):
        env = {**os.environ, "GFD_WRITE_PREALLOC": mode, "TMPDIR": d}
        cp = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "100", "--warmup", "10",
                             "--backend", "synthetic", "--no-extras"], capture_output=True, text=True, env=env,
                            check=True)
        r = json.loads(cp.stdout.strip().splitlines()[-1])
        print(f"  GFD_WRITE_PREALLOC={mode:5s} cycle p50 {r['value']:.4f} ms  write p50 "
              f"{r['phases_p50_ms']['write']:.4f} ms")


def main() -> int:
    base = sys.argv[1] if len(sys.argv) > 1 else None
    d = tempfile.mkdtemp(prefix="gfd-write-ab-", dir=base)
    try:
        print(f"directory {d} on {fs_type(d)}")
        print("syscall level (2 KB file, replace via rename):")
        syscall_ab(d)
        print("daemon writer, bench.py synthetic tree (100 steps):")
        bench_ab(d)
    finally:
        subprocess.run(["rm", "-rf", d])
    return 0


if __name__ == "__main__":
    sys.exit(main())
