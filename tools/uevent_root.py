#!/usr/bin/env python3
"""A sysfs root whose uevent counter this tool moves, for measuring the
cycles in which /sys/kernel/uevent_seqnum moved (another container
started, ...) on demand - an unprivileged box cannot make the kernel send
uevents (no loop devices, no network namespaces).

Everything else is the real thing: sys/bus, sys/class, sys/devices and
sys/module link to /sys, opt to /opt, so the daemon reads the host's PCI bus,
driver directories and KFD topology through the same kept descriptors as
with --sysfs-root=/ (the default); only sys/kernel/uevent_seqnum is a file.

    python tools/uevent_root.py DIR                # build it
    python tools/uevent_root.py DIR --bump SECONDS # build, then add 1 to the
                                                   # counter every SECONDS until killed
"""
from __future__ import annotations

import argparse
import os
import time


def build(root: str) -> str:
    os.makedirs(os.path.join(root, "sys/kernel"), exist_ok=True)
    for name in ("bus", "class", "devices", "module"):
        link = os.path.join(root, "sys", name)
        if not os.path.islink(link):
            os.symlink(f"/sys/{name}", link)
    if not os.path.islink(os.path.join(root, "opt")):
        os.symlink("/opt", os.path.join(root, "opt"))
    counter = os.path.join(root, "sys/kernel/uevent_seqnum")
    with open("/sys/kernel/uevent_seqnum") as f:
        start = f.read()
    with open(counter, "w") as f:
        f.write(start)
    return counter


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--bump", type=float, default=0)
    a = ap.parse_args()
    counter = build(a.root)
    if a.bump <= 0:
        return 0
    n = int(open(counter).read())
    while True:
        time.sleep(a.bump)
        n += 1
        with open(counter, "r+") as f:  # in place: the daemon preads a kept descriptor
            f.write(f"{n}\n")
            f.truncate()


if __name__ == "__main__":
    raise SystemExit(main())
