"""Shared by the fake `docker` and `kubectl` (this directory): start the
daemon binary the way a container runtime would start the labeler image.

There is no container runtime, cluster or network here or on the GPU box, so
tests/e2e/*.py - the counterparts of the reference's integration and e2e
scripts - run against these two stand-ins, put first on PATH:

* a container's bind mounts become symlinks under a scratch root
  (`<state>/<name>/root`) - the host's /opt a copy of its ROCm version file -
  and every path-valued GFD_* setting is re-rooted there: the daemon reads
  /sys and writes its feature file exactly where the container would;
* /sys is the host's own unless FAKE_SYSFS_ROOT names a synthetic tree (CPU
  runs); the host's /opt is FAKE_HOST_OPT or /opt;
* "the image" is the Dockerfile's runtime stage assembled offline
  (`_image.py`): the daemon starts from the image's own files, through the
  image's loader, with only the image's libraries to load; the loader's
  library trace is kept in <state>/<name>/ld.<pid>.
"""

from __future__ import annotations

import os
import shutil
import signal
import subprocess
import time
from pathlib import Path

import _image

REPO = Path(__file__).resolve().parents[3]
STATE = Path(os.environ.get("FAKE_RUNTIME_STATE", "/tmp/gfd-fake-runtime"))
PATH_ENV = ("GFD_OUTPUT_FILE", "GFD_HOST_ROOT", "GFD_CONFIG_FILE", "CONFIG_FILE", "GFD_ROCM_VERSION_FILE",
            "GFD_MACHINE_TYPE_FILE")
DEFAULT_OUTPUT = "/etc/kubernetes/node-feature-discovery/features.d/gfd"


def host_path(path: str) -> str:
    """Where a host path really is for this emulation: /etc/... lives in the
    emulated node's own directory (created on demand, as a DirectoryOrCreate
    hostPath is), /opt is FAKE_HOST_OPT if set, anything else is itself."""
    if path == "/opt" and os.environ.get("FAKE_HOST_OPT"):
        return os.environ["FAKE_HOST_OPT"]
    if path.startswith("/etc/"):
        real = STATE / "node" / path.lstrip("/")
        real.mkdir(parents=True, exist_ok=True)
        return str(real)
    return path


def start(name: str, mounts: list[tuple[str, str]], env: dict[str, str], args: list[str]) -> int:
    """Start the labeler with `mounts` (host path, container path); returns its pid."""
    croot = STATE / name / "root"
    croot.mkdir(parents=True, exist_ok=True)
    sys_root = None
    for src, dst in mounts:
        if dst == "/sys":
            if src != "/sys":
                raise SystemExit(f"fake runtime: /sys must be mounted from /sys, not {src}")
            sys_root = os.environ.get("FAKE_SYSFS_ROOT")
            continue
        link = croot / dst.lstrip("/")
        link.parent.mkdir(parents=True, exist_ok=True)
        real = host_path(src)
        if src == "/opt":
            # A symlink would be re-rooted by --host-root's path walk (it
            # follows the host's absolute links inside the mount): copy what
            # the daemon reads from the host's /opt instead.
            ver = Path(real) / "rocm" / ".info" / "version"
            if ver.exists():
                (link / "rocm" / ".info").mkdir(parents=True, exist_ok=True)
                shutil.copyfile(os.path.realpath(ver), link / "rocm" / ".info" / "version")
            else:
                link.mkdir(parents=True, exist_ok=True)
            continue
        if not Path(real).is_dir():
            raise SystemExit(f"fake runtime: mount source {real} is not a directory")
        if not link.is_symlink():
            link.symlink_to(real)
    penv = {k: v for k, v in os.environ.items() if not k.startswith(("GFD_", "FAKE_", "MIG_STRATEGY", "FAIL_ON"))}
    cenv = dict(env)
    for k in PATH_ENV:
        if k in cenv:
            cenv[k] = str(croot) + cenv[k]
    if not any(a.startswith(("--output-file", "--output=", "-o")) for a in args) and "GFD_OUTPUT_FILE" not in env:
        cenv["GFD_OUTPUT_FILE"] = str(croot) + DEFAULT_OUTPUT
    if sys_root:
        cenv["GFD_SYSFS_ROOT"] = sys_root
        cenv.setdefault("GFD_MACHINE_TYPE_FILE", sys_root + "/sys/class/dmi/id/product_name")
    argv, penv = _image.command(_image.build(), args, cenv, base=penv, trace=STATE / name / "ld")
    log = open(STATE / name / "log", "w")
    p = subprocess.Popen(argv, env=penv, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    (STATE / name / "pid").write_text(str(p.pid))
    return p.pid


def stop(name: str) -> None:
    pid_file = STATE / name / "pid"
    if not pid_file.exists():
        return
    pid = int(pid_file.read_text())
    try:
        os.kill(pid, signal.SIGTERM)
        for _ in range(100):
            try:
                if os.waitpid(pid, os.WNOHANG) != (0, 0):
                    break
            except ChildProcessError:  # not our child: poll its /proc entry
                if not Path(f"/proc/{pid}").exists():
                    break
            time.sleep(0.05)
        else:
            os.kill(pid, signal.SIGKILL)
    except ProcessLookupError:
        pass
    pid_file.unlink()
