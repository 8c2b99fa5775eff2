"""Differential harness: a long-lived daemon against fresh processes.

The daemon keeps state between its cycles that the reference, which builds
its labelers and initialises NVML anew every cycle
(cmd/gpu-feature-discovery/main.go:160, internal/lm/nvml.go:30-33), cannot
have: the amd-smi session and what it learned (handles, ASIC identity,
supported partition modes), the KFD topology of a generation, the SR-IOV
functions while no uevent was sent (and, after one, while the driver
directories and VF links are unchanged), the amdgpu module directory, open
attribute descriptors, the feature file and its swapped-out spare.  Each of those is only
correct if everything that can change it also invalidates it.

This module changes a synthetic MI355X node the way the kernel and an
administrator would - a partition or NPS switch, VFs enabled or disabled,
a GPU added or removed, the amdgpu module reloaded, a driver bound or
unbound, /opt/rocm repointed, the ROCm version file rewritten in place or
replaced, the DMI product name changed, an unrelated uevent - bumping
/sys/kernel/uevent_seqnum and the KFD topology's generation_id exactly when
the kernel would (any device or binding added or removed sends a uevent;
any change of the KFD topology rebuilds it), and compares after every change
the feature file of long-lived sessions (LongLived: one process holding
daemon sessions across every change) with that of a fresh daemon process
(`--oneshot`), byte for byte.

The node model keeps what real nodes cannot do out: VFs are enabled only on
a GIM host, whose SR-IOV PFs are bound to gim and so have no KFD node and
are invisible to amd-smi (amdgpu implements no sriov_configure), and only
on a bound PF - unbinding one disables its VFs (the PF driver's remove
does; the PCI core warns "driver left SR-IOV enabled after remove"
otherwise); TotalVFs is fixed per device; a hot-added GPU keeps the others'
identities.

Nodes are changed in place, as the kernel does: an attribute rewritten
keeps its inode, a removed device's files disappear, a reloaded module's
directory and its driver directory are new directories.
"""

from __future__ import annotations

import json
import os
import random
import shutil
import subprocess
import sys
from dataclasses import dataclass, field, replace
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from gpu_feature_discovery_amd.utils import synth  # noqa: E402

MODES = ("SPX", "DPX", "QPX", "CPX")
NPS = ("NPS1", "NPS2")
ROCM_INSTALLS = ("7.0.2", "7.1.1", "7.2.0")
MACHINES = ("WB SERVER E6-IS", "AS-8125GS-TNMR2", "G893-ZX1-AAX2", "PowerEdge XE9785")


@dataclass
class Gpu:
    bus: int
    unique: int
    serial: int
    mode: str = "SPX"
    nps: str = "NPS1"
    sriov: bool = False     # has an SR-IOV capability (TotalVFs 8: fixed by the device)
    vfs: int = 0            # VFs enabled: only on a GIM host (amdgpu cannot enable VFs)
    bound: bool = True      # bound to its driver (amdgpu, or gim for an SR-IOV PF on a GIM host)
    vf: bool = False        # an SR-IOV VF handed to this node, a guest VM


@dataclass
class Node:
    gpus: list[Gpu] = field(default_factory=list)
    driver_version: str = "6.12.12"
    gim: str | None = None
    machine: str = MACHINES[0]
    rocm_link: str = "7.2.0"                            # opt/rocm -> rocm-<this>
    rocm_text: dict = field(default_factory=lambda: {v: v for v in ROCM_INSTALLS})  # install -> version file text
    layout: str = "function"
    guest: bool = False  # a VM whose GPUs are VFs (CPU hypervisor flag set)
    seqnum: int = 4000
    generation: int = 1


def spec_of(node: Node) -> synth.NodeSpec:
    gpus = []
    for g in node.gpus:
        sriov = {"total": 8, "num": g.vfs, "vf_device": synth.MI355X_VF_DEVICE_ID} if g.sriov else None
        # On a GIM host the SR-IOV PFs are bound to gim, which creates no KFD
        # node (and amd-smi, which goes through amdgpu, does not see them).
        on_gim = g.sriov and node.gim is not None
        gpus.append(synth.GpuSpec(compute_partition=g.mode, memory_partition=g.nps, sriov=sriov, bus=g.bus,
                                  unique_id=g.unique, serial=g.serial, driver="auto" if g.bound else None,
                                  kfd=g.bound and not on_gim, vf=g.vf,
                                  available_compute="SPX, DPX, QPX, CPX" if g.nps == "NPS1" else "DPX, QPX, CPX"))
    return synth.NodeSpec(gpus=gpus, driver_version=node.driver_version, machine=node.machine,
                          partition_layout=node.layout, rocm_version_file=False, gim_version=node.gim, seed=5,
                          hypervisor=node.guest)


def _remove(p: str) -> None:
    if os.path.islink(p) or os.path.isfile(p):
        os.unlink(p)
    elif os.path.isdir(p):
        shutil.rmtree(p)


class LiveNode:
    """A synthetic node under `root`, kept in sync with a Node model."""

    def __init__(self, root: Path, node: Node):
        self.root = Path(root)
        self.node = node
        self.tree: dict[str, tuple] = {}  # what is on disk under root (the last target)
        self.root.mkdir(parents=True, exist_ok=True)
        self.apply(force_structure=True)

    def close(self) -> None:
        pass

    def _target(self) -> dict[str, tuple]:
        tree = synth.make_tree(spec_of(self.node))
        tree["opt"] = ("d", None)
        for v, text in self.node.rocm_text.items():
            tree[f"opt/rocm-{v}"] = tree[f"opt/rocm-{v}/.info"] = ("d", None)
            tree[f"opt/rocm-{v}/.info/version"] = ("f", (text + "\n").encode())
        tree["opt/rocm"] = ("l", f"rocm-{self.node.rocm_link}")
        tree["sys/kernel"] = ("d", None)  # uevent_seqnum: written by apply()
        return tree

    def apply(self, force_structure: bool = False, recreate: tuple[str, ...] = (), reset: bool = False) -> dict:
        """Bring the live tree to the model, in place; bump the counters as
        the kernel would.  `recreate`: directories that become new ones (a
        reloaded module's).  `reset`: the GPUs were reset (new KFD nodes and
        uevents even where no file changed).  Returns what changed."""
        target = self._target()
        old = self.tree

        def differs(prefix: str, structural: bool) -> bool:
            for k in {k for k in set(old) | set(target) if k.startswith(prefix) and not k.endswith("generation_id")}:
                a, b = old.get(k), target.get(k)
                if a is None or b is None or a[0] != b[0] or (a[0] == "l" and a != b):
                    return True
                if not structural and a != b:
                    return True
            return False

        kfd_changed = force_structure or reset or bool(recreate) or differs("sys/class/kfd", False)
        uevent = force_structure or reset or bool(recreate) or differs("sys/bus", True) or differs("sys/module", True)
        self.node.generation += kfd_changed
        self.node.seqnum += uevent
        target["sys/class/kfd/kfd/topology/generation_id"] = ("f", f"{self.node.generation}\n".encode())
        target["sys/kernel/uevent_seqnum"] = ("f", f"{self.node.seqnum}\n".encode())
        live = dict(old)
        for d in recreate:
            _remove(str(self.root / d))
            for k in [k for k in live if k == d or k.startswith(d + "/")]:
                del live[k]
        # Remove what the target no longer has (deepest first), then create
        # or rewrite in place what it has.
        for k in sorted(set(live) - set(target), key=lambda k: -k.count("/")):
            _remove(str(self.root / k))
        for k in sorted(target, key=lambda k: k.count("/")):
            kind, val = target[k]
            cur = live.get(k)
            if cur == target[k]:
                continue
            p = self.root / k
            if cur is not None and (cur[0] != kind or kind == "l"):
                _remove(str(p))
                cur = None
            if kind == "d":
                p.mkdir(exist_ok=True)
            elif kind == "l":
                os.symlink(val, p)
            else:
                with open(p, "r+b" if cur is not None else "wb") as f:  # in place: same inode
                    f.write(val)
                    f.truncate()
        self.tree = target
        return {"generation": kfd_changed, "uevent": uevent}

    def fake_spec(self) -> str:
        return synth.fake_amdsmi_spec(self.root, spec_of(self.node)).replace("\n", "|")


# ---------------------------------------------------------------------------
# Changes


def _free_bus(node: Node, rng: random.Random) -> int:
    used = {g.bus for g in node.gpus}
    return rng.choice([b for b in range(0x10, 0xF0, 0x10) if b not in used] or [0xF1])


def new_gpu(node: Node, rng: random.Random) -> Gpu:
    return Gpu(bus=_free_bus(node, rng), unique=rng.getrandbits(64), serial=rng.randint(10**11, 10**12 - 1),
               mode=rng.choice(MODES), nps=rng.choice(NPS))


def guest_gpu(node: Node, rng: random.Random) -> Gpu:
    """A GPU of a VM: mostly a VF, sometimes a whole GPU passed through; a VF
    that amdgpu failed to probe stays unbound."""
    g = new_gpu(node, rng)
    g.vf, g.mode, g.nps = rng.random() < 0.7, "SPX", "NPS1"
    if g.vf and rng.random() < 0.25:
        g.bound = False
    return g


def random_node(rng: random.Random) -> Node:
    if rng.random() < 0.15:
        # A guest VM: its GPUs are VFs in SPX, it runs no SR-IOV host driver.
        node = Node(machine=rng.choice(MACHINES), rocm_link=rng.choice(ROCM_INSTALLS), guest=True)
        for _ in range(rng.randint(1, 2)):
            node.gpus.append(guest_gpu(node, rng))
        return node
    node = Node(gim=rng.choice([None, "8.3.0.K"]), machine=rng.choice(MACHINES), rocm_link=rng.choice(ROCM_INSTALLS),
                layout=rng.choice(["function", "function", "shared"]))
    for _ in range(rng.randint(1, 3)):
        g = new_gpu(node, rng)
        if rng.random() < 0.4:
            g.sriov, g.vfs = True, rng.randint(0, 3) if node.gim else 0
        node.gpus.append(g)
    return node


def mutate(live: LiveNode, rng: random.Random) -> str:
    """One random change to the node, applied in place; returns its name."""
    n = live.node
    kinds = ["partition", "nps", "vfs", "gpu_add", "gpu_remove", "module_reload", "rocm_repoint", "rocm_rewrite",
             "rocm_replace", "dmi", "bind", "uevent"]
    kind = rng.choice(kinds)
    if kind in ("partition", "nps", "vfs", "gpu_remove", "bind") and not n.gpus:
        kind = "gpu_add"
    if n.guest and kind in ("partition", "nps", "vfs"):
        # A VF's modes are the host's business; what a guest sees change is
        # VFs hot-plugged, removed, probed or not.
        kind = rng.choice(["gpu_add", "gpu_remove", "bind", "uevent"]) if n.gpus else "gpu_add"
    recreate: tuple[str, ...] = ()
    reset = False
    if kind == "partition":
        g = rng.choice(n.gpus)
        g.mode = rng.choice([m for m in MODES if m != g.mode])
    elif kind == "nps":
        g = rng.choice(n.gpus)
        g.nps = "NPS2" if g.nps == "NPS1" else "NPS1"
        reset = True  # a memory-partition switch resets the GPU: new KFD nodes, uevents
    elif kind == "vfs" and n.gim is None:
        # No SR-IOV host driver: VFs cannot be enabled; the change is GIM
        # being installed (its module appears, it binds the SR-IOV PFs).
        n.gim = "8.3.0.K"
    elif kind == "vfs":
        capable = [g for g in n.gpus if g.sriov and g.bound]
        if not capable:
            g = rng.choice(n.gpus)
            g.sriov = True  # (a GPU of another SKU: as if hot-added with its capability)
            n.gpus.remove(g)
            n.gpus.append(replace(g, bus=_free_bus(n, rng), unique=rng.getrandbits(64)))
        else:
            g = rng.choice(capable)
            g.vfs = rng.choice([v for v in (0, 1, 2, 3) if v != g.vfs])
    elif kind == "gpu_add":
        n.gpus.append(guest_gpu(n, rng) if n.guest else new_gpu(n, rng))
    elif kind == "gpu_remove":
        n.gpus.pop(rng.randrange(len(n.gpus)))
    elif kind == "module_reload":
        n.driver_version = rng.choice(["6.12.12", "6.14.2", "6.16.0"])
        recreate = ("sys/module/amdgpu", "sys/bus/pci/drivers/amdgpu")
    elif kind == "rocm_repoint":
        n.rocm_link = rng.choice([v for v in ROCM_INSTALLS if v != n.rocm_link])
    elif kind == "rocm_rewrite":
        n.rocm_text[n.rocm_link] = rng.choice(["7.2.1", "7.3.0", "8.0.0", n.rocm_link + "-99"])
    elif kind == "rocm_replace":
        text = rng.choice(["7.2.2", "7.4.0", "garbage"])
        n.rocm_text[n.rocm_link] = text
        p = live.root / f"opt/rocm-{n.rocm_link}/.info/version"
        tmp = p.with_name(".version.new")
        tmp.write_text(text + "\n")
        os.replace(tmp, p)  # a new inode at the same path (a package upgrade)
    elif kind == "dmi":
        n.machine = rng.choice([m for m in MACHINES if m != n.machine])
    elif kind == "bind":
        g = rng.choice(n.gpus)
        g.bound = not g.bound
        if not g.bound:
            g.vfs = 0  # the PF driver disables SR-IOV as it unbinds
    elif kind == "uevent":
        n.seqnum += rng.randint(1, 40)  # a container's veth, a loop device...
    live.apply(recreate=recreate, reset=reset)
    return kind


def scripted_sequences() -> list[tuple[Node, list]]:
    """Fixed sequences for changes the random ones reach too rarely to guard
    (each step: a function(live) that changes the node and returns a name).
    A VM with a whole GPU passed through, to which a VF is hot-plugged that
    amdgpu does not probe, then removed; then one that amdgpu probes, then
    unbinds: only the bus shows the unbound VF (sriov/bound.h)."""
    def vm() -> Node:
        node = Node(guest=True)
        node.gpus.append(Gpu(bus=0x10, unique=0x1111, serial=10**11 + 1))
        return node

    def add_vf(bound: bool):
        def step(live: LiveNode) -> str:
            n = live.node
            n.gpus.append(Gpu(bus=0x20, unique=0x2222, serial=10**11 + 2, vf=True, bound=bound))
            live.apply()
            return "gpu_add"
        return step

    def remove_vf(live: LiveNode) -> str:
        live.node.gpus = [g for g in live.node.gpus if not g.vf]
        live.apply()
        return "gpu_remove"

    def unbind_vf(live: LiveNode) -> str:
        for g in live.node.gpus:
            if g.vf:
                g.bound = False
        live.apply()
        return "bind"

    return [(vm(), [add_vf(False), remove_vf, add_vf(True), unbind_vf, remove_vf])]


# ---------------------------------------------------------------------------
# Both sides

_SERVER = r"""
import ctypes, json, os, sys
sys.path.insert(0, sys.argv[1])
import gpu_feature_discovery_amd as gfd
g = gfd.native(); g.set_quiet(True)
fake = ctypes.CDLL(os.environ["GFD_AMDSMI_LIBRARY"])
sessions = {}
for line in sys.stdin:
    req = json.loads(line)
    op = req["op"]
    try:
        if op == "open":
            sessions[req["id"]] = g.Session(req["args"])
            res = {"ok": True}
        elif op == "close":
            sessions.pop(req["id"], None)
            res = {"ok": True}
        elif op == "stage":
            fake.fake_amdsmi_stage(req["spec"].replace("|", "\n").encode())
            res = {"ok": True}
        else:
            sessions[req["id"]].cycle(True)
            with open(req["out"]) as f:
                res = {"ok": True, "out": f.read()}
    except Exception as e:  # a cycle's error is a result to compare
        res = {"ok": False, "err": str(e)}
    sys.stdout.write(json.dumps(res) + "\n")
    sys.stdout.flush()
"""


class LongLived:
    """One process holding daemon sessions (cli::label_cycle, the daemon's
    own loop body, with the feature file written) across every change."""

    def __init__(self, fake_lib: str):
        env = {**os.environ, "GFD_AMDSMI_LIBRARY": fake_lib, "GFD_FAKE_AMDSMI_SPEC": ""}
        self.p = subprocess.Popen([sys.executable, "-c", _SERVER, str(REPO)], stdin=subprocess.PIPE,
                                  stdout=subprocess.PIPE, text=True, env=env)

    def call(self, **req) -> dict:
        self.p.stdin.write(json.dumps(req) + "\n")
        self.p.stdin.flush()
        line = self.p.stdout.readline()
        if not line:
            raise RuntimeError("long-lived session process died")
        return json.loads(line)

    def close(self) -> None:
        self.p.stdin.close()
        self.p.wait(timeout=30)


def daemon_args(root: Path, backend: str, strategy: str, out: str) -> list[str]:
    return [f"--backend={backend}", f"--sysfs-root={root}", f"--machine-type-file={root}/sys/class/dmi/id/product_name",
            f"--mig-strategy={strategy}", "--no-timestamp", f"--output-file={out}"]


def fresh(binary: str, args: list[str], out: str, env: dict) -> dict:
    """A fresh daemon process (`--oneshot`): the reference's every-cycle view."""
    if os.path.exists(out):
        os.unlink(out)
    cp = subprocess.run([binary, "--oneshot", *args], capture_output=True, text=True, env=env, timeout=60)
    if cp.returncode != 0:
        errs = [ln.split("Error: ", 1)[1] for ln in cp.stderr.splitlines() if "Error: " in ln]
        return {"ok": False, "err": errs[-1] if errs else cp.stderr[-500:]}
    with open(out) as f:
        return {"ok": True, "out": f.read()}
