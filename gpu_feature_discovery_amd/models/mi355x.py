"""Hardware model of the AMD Instinct MI355X as the daemon sees it.

One place for the device facts that synthetic trees, goldens and tests are
built from, all measured on the MI355X pool (profiles/hw_probe.md,
profiles/amdsmi_api_latency_probe.txt) rather than taken from datasheets:

* PCI identity: vendor 0x1002, PF device 0x75a3, MxGPU VF device 0x75b3,
  class 0x1200 (processing accelerator), board "AMD Instinct MI355 OAM";
* ISA gfx950 (KFD ``gfx_target_version`` 90500, amd-smi 0x950), CDNA4;
* 256 CUs in 8 XCDs (KFD ``simd_count`` 1024 at 4 SIMDs/CU, ``num_xcc`` 8);
* 309220868096 bytes of HBM3E = 294896 MiB (what amdgpu reports, a little
  under the marketed 288 GB);
* 8 GPUs per xGMI hive, 7 links per GPU;
* compute partition modes SPX/DPX/QPX/CPX (1/2/4/8 partitions of 8/4/2/1
  XCDs), memory partition modes NPS1/NPS2 on the pool (NPS4 on other
  platforms).

:func:`partition_profile` mirrors the native ``resource::partition_profile_name``
(``src/resource/device.cpp``) so tests can predict the label names of any
mode combination, e.g. ``cpx.1xcd.36gb``.  The reference's equivalent is
go-nvlib's MIG profile naming (``mig_profile.go:200-209``, ``%dg.%dgb``).
"""

from __future__ import annotations

from dataclasses import dataclass

VENDOR_ID = 0x1002
DEVICE_ID = 0x75A3
VF_DEVICE_ID = 0x75B3
PCI_CLASS = 0x120000
PRODUCT_NAME = "AMD Instinct MI355 OAM"
GFX_TARGET = "gfx950"
GFX_TARGET_VERSION = 90500  # KFD spelling
FAMILY = "cdna4"
VRAM_BYTES = 309220868096
VRAM_MIB = VRAM_BYTES >> 20  # 294896
CUS = 256
XCDS = 8
SIMDS_PER_CU = 4
HIVE_SIZE = 8
XGMI_LINKS = HIVE_SIZE - 1

PARTITIONS_PER_MODE = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
NPS_COUNT = {"NPS1": 1, "NPS2": 2, "NPS4": 4, "NPS8": 8}
POOL_MEMORY_MODES = ("NPS1", "NPS2")


@dataclass(frozen=True)
class Partition:
    """One compute partition of a GPU in a given (compute, memory) mode."""

    compute_mode: str
    memory_mode: str
    xcds: int
    compute_units: int
    memory_mib: int

    @property
    def profile(self) -> str:
        return partition_profile(self.compute_mode, self.xcds, self.memory_mib)


def partition_profile(compute_mode: str, xcds: int, memory_mib: int) -> str:
    """``<mode>.<xcds>xcd.<gb>gb`` with GB rounded to the nearest integer
    (36862 MiB -> 36gb), lower-case mode (``xcp`` if unknown); same rule as
    the daemon."""
    gb = (memory_mib + 512) // 1024
    return f"{(compute_mode or 'xcp').lower()}.{xcds}xcd.{gb}gb"


def partitions(compute_mode: str, memory_mode: str = "NPS1") -> list[Partition]:
    """The partitions one MI355X exposes in ``compute_mode``/``memory_mode``.

    Memory is split evenly over the compute partitions (each partition sees
    its share of HBM regardless of NPS mode; NPS decides locality, not
    capacity).  That is the model of upstream amdgpu's per-XCP memory
    (``KFD_XCP_MEMORY_SIZE``, reported in each partition node's KFD
    ``mem_banks``), not a measurement: the pool runs SPX/NPS1 only and
    cannot switch modes (profiles/hw_probe.md), so no partitioned MI355X has
    been observed.
    """
    n = PARTITIONS_PER_MODE[compute_mode]
    if memory_mode not in NPS_COUNT:
        raise ValueError(f"unknown memory partition mode {memory_mode!r}")
    if NPS_COUNT[memory_mode] > n:
        raise ValueError(f"{memory_mode} needs at least {NPS_COUNT[memory_mode]} compute partitions, {compute_mode} "
                         f"has {n}")
    return [Partition(compute_mode, memory_mode, XCDS // n, CUS // n, VRAM_MIB // n) for _ in range(n)]


def valid_modes() -> list[tuple[str, str]]:
    """Every (compute, memory) mode pair the model accepts."""
    return [(c, m) for c in PARTITIONS_PER_MODE for m in NPS_COUNT if NPS_COUNT[m] <= PARTITIONS_PER_MODE[c]]
