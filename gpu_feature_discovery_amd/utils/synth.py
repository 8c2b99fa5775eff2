"""Synthetic sysfs trees for MI355X nodes.

Builds the subset of ``/sys`` (plus ``/opt/rocm/.info/version``) that the
daemon's KFD-sysfs backend and SR-IOV scanner read, laid out exactly like the
MI355X pool (verified by tools/hw_probe.sh; see profiles/hw_probe.md):

* ``sys/class/kfd/kfd/topology/nodes/N/properties`` and ``mem_banks`` - one
  node per CPU socket, then one node per GPU (SPX) or per compute partition
  (DPX/QPX/CPX: 2/4/8 nodes).  A partition node's ``location_id`` follows
  ``NodeSpec.partition_layout``: ``"function"`` (upstream amdgpu on GC
  9.4.3-class parts ORs the partition index into the PCI function bits, so
  partition k of ``bb:00.0`` reports ``bb:00.k``), ``"shared"`` (older
  kernels: every partition reports the parent's location) or
  ``"distinct-ids"`` (function addresses, and every partition reports its
  own ``unique_id`` / ASIC serial - a kernel with per-XCP identities),
* ``sys/bus/pci/devices/<bdf>/...`` - product name, partition modes, VRAM,
  xGMI link table, SR-IOV attributes, configuration space,
* ``sys/module/amdgpu/version``, ``sys/class/dmi/id/product_name``.

Device identities (PCI bus numbers, unique IDs / UUIDs, serials) are random
but reproducible from ``seed``, matching the benchmark spec ("synthetic/mock
sysfs tree with random device IDs").
"""

from __future__ import annotations

import os
import random
import struct
from dataclasses import dataclass, field
from pathlib import Path

from ..models import mi355x

MI355X_DEVICE_ID = mi355x.DEVICE_ID
MI355X_VF_DEVICE_ID = mi355x.VF_DEVICE_ID
MI355X_VRAM_BYTES = mi355x.VRAM_BYTES  # 294896 MiB, as reported by amdgpu
MI355X_CUS = mi355x.CUS
MI355X_XCDS = mi355x.XCDS
PARTITIONS_PER_MODE = mi355x.PARTITIONS_PER_MODE
NPS_COUNT = mi355x.NPS_COUNT


@dataclass
class GpuSpec:
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    device_id: int = MI355X_DEVICE_ID
    product_name: str = "AMD Instinct MI355 OAM"
    vram_bytes: int = MI355X_VRAM_BYTES
    cus: int = MI355X_CUS
    xcds: int = MI355X_XCDS
    gfx_target_version: int = 90500
    # SR-IOV: None, or dict(total=8, num=4, vf_device=0x75b3)
    sriov: dict | None = None
    # True: the KFD nodes of this GPU are not readable (not allocated to the
    # container), like the other 7 GPUs on a 1-GPU pool box.
    hidden: bool = False
    # True: this GPU is an SR-IOV virtual function handed to a guest VM (VF
    # device ID, no SR-IOV capability of its own, no physfn link).
    vf: bool = False
    # Partition indices whose KFD nodes the container may read (None: all),
    # e.g. [3] for a pod that was allocated one CPX partition.
    visible_partitions: list[int] | None = None
    # PCI driver bound to the function (sys/bus/pci/drivers/<driver>/<bdf>):
    # "auto" = gim for an SR-IOV PF on a GIM host, else amdgpu; None = none
    # (a guest whose amdgpu is not loaded).
    driver: str | None = "auto"
    # Fixed identity (None: drawn from the node's seed): keeps a GPU's PCI
    # bus and ASIC serial when other GPUs are added or removed (hot-plug).
    bus: int | None = None
    unique_id: int | None = None
    # False: no KFD nodes (amdgpu does not drive the function, e.g. unbound).
    serial: int | None = None
    kfd: bool = True
    # Compute partition modes the driver offers (amdgpu narrows them under
    # some memory partition modes).
    available_compute: str = "SPX, DPX, QPX, CPX"


@dataclass
class NodeSpec:
    gpus: list[GpuSpec] = field(default_factory=list)
    cpu_sockets: int = 2
    driver_version: str = "6.12.12"
    rocm_version: str = "7.2.0"
    machine: str = "WB SERVER E6-IS"
    privileged: bool = False  # full 4 KiB config space readable
    seed: int = 0
    hive_size: int = 8  # GPUs per xGMI hive (MI355X platforms: 8)
    hypervisor: bool = False  # CPU "hypervisor" flag (running inside a VM)
    partition_layout: str = "function"  # "function" | "shared" | "distinct-ids" (see module docstring)
    rocm_version_file: bool = True  # write opt/rocm/.info/version
    gim_version: str | None = None  # SR-IOV host driver (GIM) loaded: sys/module/gim/version


# make_tree(): (root, {relative path: (kind, value)}) collecting what
# make_node would write, instead of writing it.
_sink: tuple[Path, dict] | None = None


def _record(path: Path, entry: tuple) -> None:
    root, tree = _sink
    rel = path.relative_to(root)
    for parent in list(rel.parents)[:-1]:
        tree.setdefault(str(parent), ("d", None))
    tree[str(rel)] = entry


def _mkdir(path: Path) -> None:
    if _sink:
        _record(path, ("d", None))
    else:
        path.mkdir(parents=True, exist_ok=True)


def _symlink(path: Path, target: str) -> None:
    if _sink:
        _record(path, ("l", target))
    else:
        path.symlink_to(target)


def _write(path: Path, text: str | bytes) -> None:
    if _sink:
        _record(path, ("f", text if isinstance(text, bytes) else text.encode()))
        return
    path.parent.mkdir(parents=True, exist_ok=True)
    if isinstance(text, bytes):
        path.write_bytes(text)
    else:
        path.write_text(text)


def config_space(device_id: int, sriov: dict | None, size: int) -> bytes:
    """PCI configuration space of an AMD accelerator function.

    Capability chain PM(0x48) -> PCIe(0x64) -> MSI(0xa0) -> MSI-X(0xc0);
    extended chain AER(0x100) -> ARI(0x150) -> [SR-IOV(0x200)] -> VSEC(0x300).
    ``size`` 64 models an unprivileged reader (what the pool exposes).
    """
    b = bytearray(4096)
    struct.pack_into("<HHHH", b, 0, 0x1002, device_id, 0x0407, 0x0010)
    b[0x0B] = 0x12
    struct.pack_into("<HH", b, 0x2C, 0x1002, device_id)
    b[0x34] = 0x48
    b[0x48:0x4C] = bytes([0x01, 0x64, 0x03, 0x00])
    b[0x64:0x68] = bytes([0x10, 0xA0, 0x02, 0x00])
    b[0xA0:0xA2] = bytes([0x05, 0xC0])
    b[0xC0:0xC2] = bytes([0x11, 0x00])
    after_ari = 0x200 if sriov else 0x300
    struct.pack_into("<I", b, 0x100, 0x0001 | (1 << 16) | (0x150 << 20))
    struct.pack_into("<I", b, 0x150, 0x000E | (1 << 16) | (after_ari << 20))
    if sriov:
        struct.pack_into("<I", b, 0x200, 0x0010 | (1 << 16) | (0x300 << 20))
        struct.pack_into("<H", b, 0x208, 1 if sriov.get("num", 0) else 0)
        struct.pack_into("<HHH", b, 0x20C, sriov["total"], sriov["total"], sriov.get("num", 0))
        struct.pack_into("<HH", b, 0x214, 1, 1)
        struct.pack_into("<H", b, 0x21A, sriov.get("vf_device", 0x75B3))
    struct.pack_into("<I", b, 0x300, 0x000B | (1 << 16))
    return bytes(b[:size])


def _kfd_properties(spec: GpuSpec, parts: int, location: int, render: int, unique: int, xcc: int) -> str:
    cus = spec.cus // parts
    props = {
        "cpu_cores_count": 0,
        "simd_count": cus * 4,
        "mem_banks_count": 1,
        "caches_count": 0,
        "io_links_count": 0,
        "p2p_links_count": 0,
        "cpu_core_id_base": 0,
        "simd_id_base": 2147487744 + render,
        "max_waves_per_simd": 8,
        "lds_size_in_kb": 160,
        "gds_size_in_kb": 0,
        "num_gws": 64,
        "wave_front_size": 64,
        "array_count": 32 // parts,
        "simd_arrays_per_engine": 1,
        "cu_per_simd_array": 9,
        "simd_per_cu": 4,
        "max_slots_scratch_cu": 32,
        "gfx_target_version": spec.gfx_target_version,
        "vendor_id": 4098,
        "device_id": MI355X_VF_DEVICE_ID if spec.vf else spec.device_id,
        "location_id": location,
        "domain": 0,
        "drm_render_minor": render,
        "hive_id": 6580227414736629568,
        "num_sdma_engines": max(1, 2 // parts) if parts > 1 else 2,
        "num_sdma_xgmi_engines": 14 // parts,
        "num_sdma_queues_per_engine": 8,
        "num_cp_queues": 24,
        "max_engine_clk_fcompute": 2400,
        "local_mem_size": 0,
        "fw_version": 44,
        "capability": 2889327232,
        "capability2": 1,
        "debug_prop": 1494,
        "sdma_fw_version": 14,
        "unique_id": unique,
        "num_xcc": xcc,
        "max_engine_clk_ccompute": 5008,
    }
    return "".join(f"{k} {v}\n" for k, v in props.items())


def make_node(root: str | os.PathLike, spec: NodeSpec) -> Path:
    """Materialise ``spec`` under ``root``; returns the root path."""
    root = Path(root)
    rng = random.Random(spec.seed)
    topo = root / "sys/class/kfd/kfd/topology"
    _write(topo / "generation_id", "1\n")
    _write(root / "sys/module/amdgpu/version", spec.driver_version + "\n")
    _write(root / "sys/module/amdgpu/initstate", "live\n")  # a loadable module's
    if spec.gim_version:
        _write(root / "sys/module/gim/version", spec.gim_version + "\n")
    if spec.partition_layout not in ("function", "shared", "distinct-ids"):
        raise ValueError(f"unknown partition_layout {spec.partition_layout!r}")
    if spec.rocm_version_file:
        _write(root / "opt/rocm/.info/version", spec.rocm_version + "\n")
    _write(root / "sys/class/dmi/id/product_name", spec.machine + "\n")
    flags = "fpu vme de pse tsc msr pae mce cx8 apic sep mtrr" + (" hypervisor" if spec.hypervisor else "") + " lahf_lm"
    _write(root / "proc/cpuinfo", "processor\t: 0\nvendor_id\t: AuthenticAMD\nmodel name\t: AMD EPYC 9575F 64-Core "
           f"Processor\nflags\t\t: {flags}\n\n")
    _mkdir(root / "sys/bus/pci/devices")

    node = 0
    for s in range(spec.cpu_sockets):
        _write(topo / f"nodes/{node}/properties",
               f"cpu_cores_count 128\nsimd_count 0\nmem_banks_count 1\ncpu_core_id_base {128 * s}\n"
               "gfx_target_version 0\nvendor_id 0\ndevice_id 0\nlocation_id 0\n")
        _write(topo / f"nodes/{node}/mem_banks/0/properties", "heap_type 0\nsize_in_bytes 1622942375936\n")
        node += 1

    buses = rng.sample(range(0x10, 0xF0), len(spec.gpus))
    n_gpus = len(spec.gpus)
    render = 128
    for gi, g in enumerate(spec.gpus):
        parts = PARTITIONS_PER_MODE[g.compute_partition]
        bus = buses[gi] if g.bus is None else g.bus
        location = bus << 8
        bdf = f"0000:{bus:02x}:00.0"
        unique = rng.getrandbits(64)
        if g.unique_id is not None:
            unique = g.unique_id
        xcc = g.xcds // parts
        node_mem = g.vram_bytes // parts
        for p in range(parts):
            ndir = topo / f"nodes/{node}"
            # kfd_topology.c: location_id = pci_dev_id | xcp node id.
            node_location = location | p if spec.partition_layout != "shared" and parts > 1 else location
            node_unique = unique ^ (p + 1) if spec.partition_layout == "distinct-ids" and parts > 1 else unique
            if not g.kfd:
                node -= 1  # no node of its own: the next GPU's take these ids
            elif g.hidden or (g.visible_partitions is not None and p not in g.visible_partitions):
                # Unreadable: the kernel returns EPERM; a directory named
                # `properties` makes every read fail the same way (EISDIR).
                _mkdir(ndir / "properties")
            else:
                _write(ndir / "properties", _kfd_properties(g, parts, node_location, render, node_unique, xcc))
                _write(ndir / "mem_banks/0/properties", f"heap_type 1\nsize_in_bytes {node_mem}\nflags 0\nwidth 8192\n")
                _write(ndir / "gpu_id", f"{rng.randint(1000, 65535)}\n")
            node += 1
            render += 1
        d = root / "sys/bus/pci/devices" / bdf
        device_id = MI355X_VF_DEVICE_ID if g.vf else g.device_id
        _write(d / "vendor", "0x1002\n")
        _write(d / "device", f"0x{device_id:04x}\n")
        _write(d / "subsystem_vendor", "0x1002\n")
        _write(d / "subsystem_device", f"0x{device_id:04x}\n")
        _write(d / "class", "0x120000\n")
        _write(d / "revision", "0x00\n")
        _write(d / "product_name", g.product_name + "\n")
        _write(d / "current_compute_partition", g.compute_partition + "\n")
        _write(d / "available_compute_partition", g.available_compute + "\n")
        _write(d / "current_memory_partition", g.memory_partition + "\n")
        _write(d / "available_memory_partition", "NPS1, NPS2\n")
        _write(d / "mem_info_vram_total", f"{g.vram_bytes}\n")
        _write(d / "unique_id", f"{unique:016x}\n")
        serial = rng.randint(10**11, 10**12 - 1)
        _write(d / "serial_number", f"{serial if g.serial is None else g.serial}\n")
        # Every GPU sits in an 8-GPU xGMI hive whether or not the other GPUs
        # are visible to this container (measured: 7 peers on a 1-GPU box).
        peers = ["01"] * spec.hive_size
        peers[gi % spec.hive_size] = "00"
        _write(d / "xgmi_num_links", " ".join(peers) + " \n")
        sriov = g.sriov or {}
        if not g.vf:
            _write(d / "sriov_totalvfs", f"{sriov.get('total', 1)}\n")
            _write(d / "sriov_numvfs", f"{sriov.get('num', 0)}\n")
        _write(d / "config", config_space(device_id, g.sriov, 4096 if spec.privileged else 64))
        if spec.privileged:
            # Per-partition resources of the current mode (amdgpu_xcp.c); mode
            # 0400 on real nodes, so only a privileged reader sees them.
            # Illustrative counts: 4 decoders / 32 JPEG engines per GPU.
            for res, total in (("xcc", g.xcds), ("dma", 16), ("dec", 4), ("jpeg", 32)):
                _write(d / f"compute_partition_config/{res}/num_inst", f"{max(1, total // parts)}\n")
                _write(d / f"compute_partition_config/{res}/num_shared", f"{max(1, parts // total)}\n")
        driver = g.driver
        if driver == "auto":
            driver = "gim" if g.sriov and spec.gim_version else "amdgpu"
        _write(d / "uevent", (f"DRIVER={driver}\n" if driver else "") +
               f"PCI_CLASS=120000\nPCI_ID=1002:{device_id:04X}\nPCI_SUBSYS_ID=1002:{device_id:04X}\n"
               f"PCI_SLOT_NAME={bdf}\nMODALIAS=pci:v00001002d0000{device_id:04X}sv00001002sd0000{device_id:04X}"
               "bc12sc00i00\n")
        if driver:
            drv = root / "sys/bus/pci/drivers" / driver
            for f in ("bind", "unbind", "new_id", "remove_id", "uevent"):
                _write(drv / f, "")
            _symlink(drv / bdf, f"../../devices/{bdf}")
        for v in range(sriov.get("num", 0)):
            vf_bdf = f"0000:{bus:02x}:00.{v + 1}"
            vd = root / "sys/bus/pci/devices" / vf_bdf
            _write(vd / "vendor", "0x1002\n")
            _write(vd / "device", f"0x{sriov.get('vf_device', 0x75B3):04x}\n")
            _write(vd / "class", "0x120000\n")
            _write(vd / "config", config_space(sriov.get("vf_device", 0x75B3), None, 4096 if spec.privileged else 64))
            _symlink(vd / "physfn", f"../{bdf}")
            _symlink(d / f"virtfn{v}", f"../{vf_bdf}")
    # An unrelated non-AMD PCI function (the scanner must skip it).
    other = root / "sys/bus/pci/devices/0000:00:00.0"
    _write(other / "vendor", "0x1022\n")
    _write(other / "class", "0x060000\n")
    _write(other / "config", b"\x22\x10" + bytes(62))
    return root


def make_tree(spec: NodeSpec) -> dict[str, tuple]:
    """What make_node(root, spec) would write, without writing it:
    {path relative to the root: ("f", bytes) | ("l", link target) | ("d", None)}."""
    global _sink
    root = Path("/synthetic-node")
    _sink = (root, {})
    try:
        make_node(root, spec)
        return _sink[1]
    finally:
        _sink = None


def make_mi355x_node(root: str | os.PathLike, n_gpus: int = 8, compute_partition: str = "SPX",
                     memory_partition: str = "NPS1", seed: int = 0, hidden: int = 0, **kwargs) -> Path:
    """An N-GPU MI355X node; the last ``hidden`` GPUs are not readable."""
    gpus = [GpuSpec(compute_partition=compute_partition, memory_partition=memory_partition,
                    hidden=i >= n_gpus - hidden) for i in range(n_gpus)]
    return make_node(root, NodeSpec(gpus=gpus, seed=seed, **kwargs))


def fake_amdsmi_spec(root: str | os.PathLike, spec: NodeSpec, latency_us: int = 0) -> str:
    """The scriptable fake amd-smi (tests/fake_amdsmi) configured as amd-smi
    would see the node ``make_node(root, spec)`` built: same PCI addresses,
    partition layout and KFD nodes, one line per readable GPU."""
    root = Path(root)
    bdfs = "shared" if spec.partition_layout == "shared" else "function"
    lines = [f"partition_bdf={bdfs}", "sockets=slot"]
    if spec.partition_layout == "distinct-ids":
        lines.append("partition_serials=distinct")
    if latency_us:
        lines.append(f"latency_us={latency_us}")
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    node = spec.cpu_sockets
    gpu_bdfs = sorted(p.name for p in (root / "sys/bus/pci/devices").iterdir()
                      if (p / "current_compute_partition").exists())
    # make_node assigns buses in GPU order; recover each GPU's address from
    # its first partition node's location_id.
    for g in spec.gpus:
        if not g.kfd:
            continue  # no KFD nodes: amd-smi does not see it either
        parts = PARTITIONS_PER_MODE[g.compute_partition]
        first = None
        for p in range(parts):
            props = kfd / str(node + p) / "properties"
            if props.is_file():
                first = first or props
        if g.hidden or first is None:
            node += parts
            continue
        loc = int(next(ln.split()[1] for ln in first.read_text().splitlines() if ln.startswith("location_id")))
        bdf = f"0000:{loc >> 8:02x}:00.0"
        assert bdf in gpu_bdfs
        fields = [f"bdf={bdf}", f"mode={g.compute_partition}", f"nps={g.memory_partition}", f"parts={parts}",
                  f"name={g.product_name}", f"cus={g.cus // parts}", f"xcds={g.xcds // parts}",
                  f"vram_mib={(g.vram_bytes // parts) >> 20}", f"kfd_base={node}"]
        # amdgpu's own classification (amdgpu_detect_virtualization), which
        # amd-smi reports: a VF is a guest, a PF with VFs enabled the host, a
        # whole GPU in a VM passthrough (AMDSMI_VIRTUALIZATION_MODE_*).
        virt = 3 if g.vf else 2 if (g.sriov or {}).get("num", 0) > 0 else 4 if spec.hypervisor else 1
        fields.append(f"virt={virt}")
        if g.visible_partitions is not None:
            fields.append("visible=" + ",".join(map(str, g.visible_partitions)))
        lines.append(";".join(fields))
        node += parts
    return "\n".join(lines)
