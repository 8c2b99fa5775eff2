#!/usr/bin/env python3
"""Build a sysfs root that shows all 8 GPUs of the host to the KFD-sysfs
backend, for 1/2/4/8-GPU measurements on a one-GPU box.

On the pool a box is one GPU of an 8xMI355X host.  Every GPU's amdgpu PCI
attributes are readable (sysfs is not namespaced), but the KFD topology
nodes of the seven GPUs not allocated to the container are not (EPERM).
This root therefore:

* links ``sys/bus/pci/devices``, ``sys/kernel/uevent_seqnum``,
  ``sys/class/dmi`` and ``sys/module`` to the real sysfs - every per-cycle
  attribute read is a live read of a real MI355X's driver attributes,
  through the same kept-open descriptors as in production;
* writes one KFD topology node per GPU whose properties are the allocated
  GPU's real properties with that GPU's PCI location (only read when the
  topology generation changes, i.e. once).

    python tools/hybrid_root.py DIR   # prints the number of GPUs
"""

from __future__ import annotations

import glob
import os
import sys


def main() -> int:
    root = sys.argv[1]
    pci = "/sys/bus/pci/devices"
    gpus = []
    for d in sorted(os.listdir(pci)):
        try:
            vendor = open(f"{pci}/{d}/vendor").read().strip()
            cls = open(f"{pci}/{d}/class").read().strip()
        except OSError:
            continue
        if vendor == "0x1002" and cls.startswith("0x12") and os.path.exists(f"{pci}/{d}/mem_info_vram_total"):
            gpus.append(d)
    template = None
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        try:
            text = open(p).read()
        except OSError:
            continue
        if "\nsimd_count 0\n" not in text and "gfx_target_version" in text and "simd_count" in text:
            template = text
            break
    if not template or not gpus:
        print("no readable GPU KFD node or no GPUs", file=sys.stderr)
        return 1
    os.makedirs(f"{root}/sys/bus/pci", exist_ok=True)
    os.makedirs(f"{root}/sys/kernel", exist_ok=True)
    os.makedirs(f"{root}/sys/class", exist_ok=True)
    for link, target in (("sys/bus/pci/devices", pci), ("sys/kernel/uevent_seqnum", "/sys/kernel/uevent_seqnum"),
                         ("sys/class/dmi", "/sys/class/dmi"), ("sys/module", "/sys/module")):
        if not os.path.lexists(f"{root}/{link}"):
            os.symlink(target, f"{root}/{link}")
    topo = f"{root}/sys/class/kfd/kfd/topology"
    os.makedirs(f"{topo}/nodes/0", exist_ok=True)
    open(f"{topo}/generation_id", "w").write("1\n")
    open(f"{topo}/nodes/0/properties", "w").write("cpu_cores_count 128\nsimd_count 0\ngfx_target_version 0\n")
    for i, bdf in enumerate(gpus):
        dom, bus, devfn = bdf.split(":")
        dev, fn = devfn.split(".")
        loc = (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)
        lines = []
        for line in template.splitlines():
            k = line.split(" ", 1)[0]
            if k == "location_id":
                line = f"location_id {loc}"
            elif k == "domain":
                line = f"domain {int(dom, 16)}"
            elif k == "unique_id":
                line = f"unique_id {0x5eed0000 + i}"
            lines.append(line)
        os.makedirs(f"{topo}/nodes/{i + 1}", exist_ok=True)
        open(f"{topo}/nodes/{i + 1}/properties", "w").write("\n".join(lines) + "\n")
    rocm = "/opt/rocm/.info/version"
    if os.path.exists(rocm):
        os.makedirs(f"{root}/opt/rocm/.info", exist_ok=True)
        open(f"{root}/opt/rocm/.info/version", "w").write(open(rocm).read())
    os.makedirs(f"{root}/proc", exist_ok=True)
    if not os.path.lexists(f"{root}/proc/cpuinfo"):
        os.symlink("/proc/cpuinfo", f"{root}/proc/cpuinfo")
    print(len(gpus))
    return 0


if __name__ == "__main__":
    sys.exit(main())
