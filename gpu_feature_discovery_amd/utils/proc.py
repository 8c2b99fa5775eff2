"""Wall time of a child process from spawn to exit, without the parent's
polling in the way.

``subprocess.run(..., timeout=T)`` waits for the child by polling with
sleeps of 0.5, 1, 2, 4, ... ms (CPython's ``Popen._wait`` with a timeout), so
a process that takes 3 ms is observed at 3.5 or 7.5 ms and one of 30 ms at
31.5 or 63.5 ms - the bimodal 7.56 / 64.3 ms Job-mode numbers of round 1 were
these poll boundaries.  ``subprocess.run`` also forks the whole interpreter
(~1 ms for ``/bin/true`` with the timeout, 0.27 ms without).  Here the child
is started with ``posix_spawn`` (vfork) and reaped with a blocking
``waitpid``; a watchdog thread kills it if it outlives ``timeout``.
"""

from __future__ import annotations

import os
import signal
import threading
import time

__all__ = ["spawn_wait_ms", "gpu_holds"]


def spawn_wait_ms(argv: list[str], timeout: float = 60.0, env: dict | None = None) -> float:
    """Run ``argv`` (stdout/stderr to /dev/null) and return its wall time in
    ms, spawn to exit.  Raises RuntimeError if it fails or times out."""
    actions = [(os.POSIX_SPAWN_OPEN, 1, os.devnull, os.O_WRONLY, 0),
               (os.POSIX_SPAWN_OPEN, 2, os.devnull, os.O_WRONLY, 0)]
    path = argv[0]
    t0 = time.perf_counter_ns()
    pid = os.posix_spawn(path, argv, os.environ if env is None else env, file_actions=actions)
    timed_out = threading.Event()

    def kill():
        timed_out.set()
        try:
            os.kill(pid, signal.SIGKILL)
        except ProcessLookupError:
            pass

    watchdog = threading.Timer(timeout, kill)
    watchdog.start()
    try:
        _, status = os.waitpid(pid, 0)
    finally:
        watchdog.cancel()
    ms = (time.perf_counter_ns() - t0) / 1e6
    if timed_out.is_set():
        raise RuntimeError(f"{argv[0]} timed out after {timeout} s")
    if os.waitstatus_to_exitcode(status) != 0:
        raise RuntimeError(f"{' '.join(argv)} exited with {os.waitstatus_to_exitcode(status)}")
    return ms


def gpu_holds(pid: int) -> dict:
    """What process ``pid`` holds on the GPU right now: its descriptors of
    /dev/kfd or /dev/dri/* (``readlink /proc/<pid>/fd/*``), its memory maps of
    them, and whether KFD lists it as a process (/sys/class/kfd/kfd/proc/<pid>:
    a registered KFD process, which amdgpu counts when it refuses a partition
    switch).  Also every descriptor, for the record."""
    fds = {}
    fd_dir = f"/proc/{pid}/fd"
    for name in sorted(os.listdir(fd_dir), key=int):
        try:
            fds[name] = os.readlink(f"{fd_dir}/{name}")
        except OSError:
            pass
    device = {k: v for k, v in fds.items() if v == "/dev/kfd" or v.startswith("/dev/dri/")}
    try:
        with open(f"/proc/{pid}/maps") as f:
            maps = [ln.strip() for ln in f if "/dev/kfd" in ln or "/dev/dri/" in ln]
    except OSError:
        maps = []
    return {"device_fds": device, "device_maps": maps, "kfd_process": os.path.exists(f"/sys/class/kfd/kfd/proc/{pid}"),
            "fds": fds}
