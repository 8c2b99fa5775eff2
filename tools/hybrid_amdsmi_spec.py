#!/usr/bin/env python3
"""The fake libamd_smi's node spec (tests/fake_amdsmi, GFD_FAKE_AMDSMI_SPEC:
'|' between lines) for the host's real MI355X: one GPU per AMD
accelerator-class function in SPX/NPS1 with amdgpu's VRAM attribute, at its
real PCI address, so the amd-smi backend reads each one's live amdgpu attributes.

    python tools/hybrid_amdsmi_spec.py [LATENCY_US]
"""

import os
import sys


def main() -> int:
    pci = "/sys/bus/pci/devices"
    lines = ["partition_bdf=function", "sockets=slot"]
    if len(sys.argv) > 1 and sys.argv[1] != "0":
        lines.append(f"latency_us={sys.argv[1]}")
    n = 0
    for d in sorted(os.listdir(pci)):
        try:
            vendor = open(f"{pci}/{d}/vendor").read().strip()
            cls = open(f"{pci}/{d}/class").read().strip()
            vram = int(open(f"{pci}/{d}/mem_info_vram_total").read())
        except (OSError, ValueError):
            continue
        if vendor != "0x1002" or not cls.startswith("0x12"):
            continue
        try:  # SPX/NPS1 only: that is how the spec line below describes the GPU
            modes = (open(f"{pci}/{d}/current_compute_partition").read().strip(),
                     open(f"{pci}/{d}/current_memory_partition").read().strip())
        except OSError:
            modes = ("SPX", "NPS1")
        if modes != ("SPX", "NPS1"):
            continue
        n += 1
        lines.append(f"bdf={d};mode=SPX;nps=NPS1;parts=1;name=AMD Instinct MI355X;cus=256;xcds=8;"
                     f"vram_mib={vram >> 20};kfd_base={n}")
    if not n:
        print("no MI355X found", file=sys.stderr)
        return 1
    print("|".join(lines))
    return 0


if __name__ == "__main__":
    sys.exit(main())
