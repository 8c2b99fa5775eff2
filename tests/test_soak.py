"""Long-running daemon checks: no memory or file-descriptor growth.

The reference runs forever as a DaemonSet and has no such test; a daemon that
keeps a library session and caches across cycles must prove it does not leak.
The daemon is run in loop mode with a 1 ms interval (thousands of cycles),
reloaded with SIGHUP part-way (manager, SR-IOV scanner and amd-smi session
rebuilt), and its RSS and open descriptors are compared between an early
sample (after warm-up) and the end.  Meanwhile a reader opens and reads the
feature file back to back, as NFD does once a minute: every read must be a
whole label set, and the daemon must survive the write-lease breaks those
opens cause.
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import threading
import time

import pytest

from conftest import has_amd_gpu
from gpu_feature_discovery_amd.utils import synth


def _rss_kib(pid: int) -> int:
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    return 0


def _fds(pid: int, out: str) -> tuple[int, int]:
    # Minimum over a short window: a cycle in flight holds transient
    # descriptors (the temp output file, an amd-smi device node), a leak
    # raises the floor.  The window must catch the daemon between cycles at
    # least once (see the per-cycle interval below).  The feature file and
    # the one the last write swapped out to gfd-tmp/, both kept open by
    # design (src/lm/writer.cpp Slot), are counted apart: a write swaps their
    # names, so which name a readlink sees depends on timing, not on leaks.
    # Returns (floor without them, most of them).
    # A descriptor closed between the listing and its readlink still counts:
    # skipping it let a sample taken while a re-read swaps descriptors (new
    # ones opened after the listing, old ones closed before the readlink)
    # dip below the floor.
    n, kept = [], []
    for _ in range(40):
        fds = os.listdir(f"/proc/{pid}/fd")
        k = 0
        for fd in fds:
            try:
                link = os.readlink(f"/proc/{pid}/fd/{fd}")
            except OSError:  # closed between listdir and readlink
                continue
            k += "/gfd-tmp/" in link or (bool(out) and link.split(" (deleted)")[0] == out)
        n.append(len(fds) - k)
        kept.append(k)
        time.sleep(0.01)
    return min(n), max(kept)


# NFD's side of the file, far more often than NFD: open, read, close - and
# every read must be a whole label set.  Each open can race the daemon's
# exchange and break its write lease on the swapped-out file
# (src/lm/writer.cpp).  A process of its own: a reader thread here would
# hold the GIL against the descriptor sampling above and skew its floor.
# Stops when its stdin closes; prints its counts.
_READER = r"""
import json, select, sys
out, reads, bad = sys.argv[1], 0, []
while not select.select([sys.stdin], [], [], 0)[0]:
    for _ in range(100):
        try:
            with open(out, "rb") as f:
                data = f.read()
        except FileNotFoundError:
            continue
        reads += 1
        if not data.endswith(b"\n") or b"amd.com/gpu.count=" not in data:
            bad.append(data[-80:].decode(errors="replace"))
print(json.dumps({"reads": reads, "bad": bad[:5]}))
"""


def soak(binary: str, args: list[str], seconds: float, hup_at: float | None = None, interval: str = "1ms") -> dict:
    p = subprocess.Popen([binary, f"--sleep-interval={interval}", "--trace-timing", *args], stdout=subprocess.DEVNULL,
                         stderr=subprocess.PIPE, text=True)
    cycles = [0]
    reloads = [0]
    tail: list[str] = []

    def reader():
        for line in p.stderr:
            if "Timing:" in line:
                cycles[0] += 1
            elif "Received SIGHUP" in line:
                reloads[0] += 1
            tail.append(line)
            del tail[:-20]

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    out = next((a.split("=", 1)[1] for a in args if a.startswith("--output-file=")), "")
    rd = subprocess.Popen([sys.executable, "-c", _READER, out], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    reads = {"reads": 0, "bad": ["reader did not report"]}
    try:
        deadline = time.monotonic() + 60
        while cycles[0] < 200 and time.monotonic() < deadline and p.poll() is None:
            time.sleep(0.05)
        assert p.poll() is None, "".join(tail)
        rss0, (fd0, kept0), c0 = _rss_kib(p.pid), _fds(p.pid, os.path.abspath(out) if out else ""), cycles[0]
        t0 = time.monotonic()
        hupped = False
        last_note = t0
        while time.monotonic() - t0 < seconds and p.poll() is None:
            if hup_at is not None and not hupped and time.monotonic() - t0 >= hup_at:
                p.send_signal(signal.SIGHUP)
                hupped = True
            if time.monotonic() - last_note >= 30:  # a long soak shows it is alive (pytest -s)
                last_note = time.monotonic()
                print(f"soak: {cycles[0] - c0} cycles, RSS {_rss_kib(p.pid)} KiB", flush=True)
            time.sleep(0.05)
        assert p.poll() is None, "".join(tail)
        rss1, (fd1, kept1), c1 = _rss_kib(p.pid), _fds(p.pid, os.path.abspath(out) if out else ""), cycles[0]
        # Files in gfd-tmp/: the old feature file kept for the next write
        # (and, in a write that could not reuse it, the one being made).
        tmp_files = sum(len(fs) for _, _, fs in os.walk(os.path.join(os.path.dirname(out), "gfd-tmp"))) if out else 0
    finally:
        try:
            reads = json.loads(rd.communicate(input="", timeout=30)[0])  # closes its stdin
        except (subprocess.TimeoutExpired, ValueError):
            rd.kill()
            rd.wait()
        p.send_signal(signal.SIGTERM)
        try:
            rc = p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            rc = p.wait()
        t.join(timeout=10)
    return {"rc": rc, "rss0": rss0, "rss1": rss1, "fd0": fd0, "fd1": fd1, "kept": max(kept0, kept1), "tmp_files": tmp_files, "cycles": c1 - c0, "reloads": reloads[0],
            "reads": reads["reads"], "bad_reads": reads["bad"][:5], "tail": "".join(tail)}


def _assert_steady(r: dict, min_cycles: int):
    assert r["rc"] == 0, r["tail"]  # alive to the end (a lease break does not kill it) and clean exit
    assert r["cycles"] >= min_cycles, r
    assert r["reads"] > 100 and not r["bad_reads"], (r["reads"], r["bad_reads"])
    # +1: the ROCm version's directory watch (fs::DirWatch) creates the
    # process's one inotify instance at its first successful arm; while the
    # user's inotify instances are used up (a parallel test run spawns many
    # daemons) the daemon looks the version up by path instead and arms
    # later, possibly after the first sample.  A leak per cycle would show as
    # hundreds over these thousands of cycles.
    assert r["fd1"] <= r["fd0"] + 1, f"file descriptors grew {r['fd0']} -> {r['fd1']}"
    assert r["kept"] <= 3, f"{r['kept']} feature files open (two kept by design, one being made)"
    assert r["tmp_files"] <= 2, f"{r['tmp_files']} files in gfd-tmp/: old feature files are not being reused"
    # Allocator noise only: a leak of even 100 bytes/cycle over thousands of
    # cycles would exceed this.  (Under ASan freed memory sits in its
    # quarantine, and LeakSanitizer checks leaks at exit instead.)
    assert os.environ.get("GFD_SANITIZED") or r["rss1"] - r["rss0"] <= 1024, f"RSS grew {r['rss0']} -> {r['rss1']} KiB over {r['cycles']} cycles"


def test_soak_sysfs_backend_no_growth(binary, tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=8)
    out = tmp_path / "out" / "gfd"
    r = soak(binary, ["--backend=sysfs", f"--sysfs-root={root}", f"--output-file={out}",
                      f"--machine-type-file={root}/sys/class/dmi/id/product_name"], seconds=6, hup_at=3)
    _assert_steady(r, min_cycles=1000)
    assert r["reloads"] == 1, r["tail"]
    assert not out.exists()  # removed on exit in loop mode


@pytest.mark.gpu
@pytest.mark.skipif(not has_amd_gpu(), reason="no /dev/kfd")
@pytest.mark.parametrize("session", ["persistent", "per-cycle"])
def test_soak_amdsmi_backend_no_growth(binary, tmp_path, session):
    # GFD_SOAK_SECONDS stretches the run for release qualification.
    seconds = float(os.environ.get("GFD_SOAK_SECONDS", "20"))
    out = tmp_path / "gfd"
    # per-cycle pays ~25 ms of amdsmi_init (which holds descriptors) every
    # cycle: with a 1 ms interval the daemon is between cycles 4% of the time
    # and the descriptor floor is caught only by luck; 10 ms makes it ~28%.
    per_cycle = session == "per-cycle"
    r = soak(binary, ["--backend=amdsmi", f"--amdsmi-session={session}", f"--output-file={out}"], seconds=seconds,
             hup_at=seconds / 2, interval="10ms" if per_cycle else "1ms")
    _assert_steady(r, min_cycles=int(seconds * (15 if per_cycle else 200)))
    assert r["reloads"] == 1, r["tail"]
    print(f"soak[{session}]: {r['cycles']} cycles in {seconds:.0f}s, RSS {r['rss0']} -> {r['rss1']} KiB, "
          f"fds {r['fd0']} -> {r['fd1']} (+ up to {r['kept']} feature files), {r['reads']} reads of the file")
