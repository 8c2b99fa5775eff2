"""Both hardware backends label the same node identically.

On the MI355X pool this is checked on a real (SPX) GPU
(tests/test_gpu.py::test_label_sets_identical_across_backends).  Compute
partitions cannot be switched there, so partitioned nodes are checked here:
a synthetic sysfs tree read by the KFD-sysfs backend, and the scriptable
fake amd-smi configured with the same GPUs (same PCI addresses, partition
layout, KFD nodes) read by the amd-smi backend over the same tree - the
labels must be byte-identical, under both partition address layouts and
with and without the root-only partition resource files.
"""

from __future__ import annotations

import pytest

from conftest import run_daemon
from gpu_feature_discovery_amd import BUILD_DIR
from gpu_feature_discovery_amd.utils import golden, synth

FAKE = BUILD_DIR / "libfake_amdsmi.so"


CASES = {
    "spx": dict(mode="SPX", nps="NPS1", strategy="none", n=2),
    "cpx-single": dict(mode="CPX", nps="NPS1", strategy="single", n=2),
    "cpx-mixed": dict(mode="CPX", nps="NPS1", strategy="mixed", n=2),
    "dpx-nps2-mixed": dict(mode="DPX", nps="NPS2", strategy="mixed", n=2),
    "qpx-single": dict(mode="QPX", nps="NPS1", strategy="single", n=1),
}


@pytest.mark.skipif(not FAKE.exists(), reason="libfake_amdsmi.so not built")
@pytest.mark.parametrize("privileged", [False, True], ids=["pod", "privileged"])
@pytest.mark.parametrize("layout", ["function", "shared", "distinct-ids"])
@pytest.mark.parametrize("case", list(CASES))
def test_amdsmi_and_sysfs_backends_label_identically(binary, tmp_path, case, layout, privileged):
    c = CASES[case]
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(compute_partition=c["mode"], memory_partition=c["nps"])
                                for _ in range(c["n"])],
                          partition_layout=layout, privileged=privileged, seed=21)
    root = synth.make_node(tmp_path / "root", spec)
    outs = {}
    for backend in ("sysfs", "amdsmi"):
        out = tmp_path / f"gfd-{backend}"
        env = {"GFD_AMDSMI_LIBRARY": str(FAKE), "GFD_FAKE_AMDSMI_SPEC": synth.fake_amdsmi_spec(root, spec).replace("\n", "|")}
        run_daemon(binary, "--oneshot", "--no-timestamp", f"--backend={backend}", f"--sysfs-root={root}",
                   f"--machine-type-file={root}/sys/class/dmi/id/product_name", f"--mig-strategy={c['strategy']}",
                   f"--output-file={out}", env=env, check=True)
        outs[backend] = out.read_text()
    assert outs["amdsmi"] == outs["sysfs"]
    labels = golden.parse_labels(outs["sysfs"])
    if c["mode"] != "SPX":
        key = "amd.com/gpu" if c["strategy"] == "single" else next(
            k.rsplit(".", 1)[0] for k in labels if k.startswith("amd.com/partition-") and k.endswith(".count"))
        assert (f"{key}.engines.decoder" in labels) == privileged
        assert f"{key}.engines.dma" in labels


@pytest.mark.skipif(not FAKE.exists(), reason="libfake_amdsmi.so not built")
@pytest.mark.parametrize("layout", ["function", "shared", "distinct-ids"])
def test_backends_agree_on_one_visible_partition(binary, tmp_path, layout):
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(compute_partition="CPX", visible_partitions=[5])],
                          partition_layout=layout, seed=22)
    root = synth.make_node(tmp_path / "root", spec)
    outs = {}
    for backend in ("sysfs", "amdsmi"):
        out = tmp_path / f"gfd-{backend}"
        env = {"GFD_AMDSMI_LIBRARY": str(FAKE), "GFD_FAKE_AMDSMI_SPEC": synth.fake_amdsmi_spec(root, spec).replace("\n", "|")}
        run_daemon(binary, "--oneshot", "--no-timestamp", f"--backend={backend}", f"--sysfs-root={root}",
                   f"--machine-type-file={root}/sys/class/dmi/id/product_name", "--mig-strategy=single",
                   f"--output-file={out}", env=env, check=True)
        outs[backend] = out.read_text()
    assert outs["amdsmi"] == outs["sysfs"]
    assert golden.parse_labels(outs["sysfs"])["amd.com/gpu.count"] == "1"


@pytest.mark.skipif(not FAKE.exists(), reason="libfake_amdsmi.so not built")
@pytest.mark.parametrize("layout", ["function", "shared", "distinct-ids"])
@pytest.mark.parametrize("case", ["spx", "cpx-single", "dpx-nps2-mixed"])
def test_amdsmi_without_libdrm_labels_identically(binary, tmp_path, case, layout):
    """amd-smi without libdrm_amdgpu (a slim image), as measured on the pool
    with the library hidden (tests/test_gpu.py::
    test_amdsmi_without_libdrm_labels_identically): asic_info and the
    virtualization query return NOT_SUPPORTED, the BDF query returns garbage
    with success, the partition profile table lists SPX only.  The backend
    takes each processor's address and identity from its KFD node, the
    virtualization mode and partition modes from the driver's sysfs state;
    the feature file must equal the KFD-sysfs backend's."""
    c = CASES[case]
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(compute_partition=c["mode"], memory_partition=c["nps"])
                                for _ in range(c["n"])], partition_layout=layout, seed=23)
    root = synth.make_node(tmp_path / "root", spec)
    fake_spec = synth.fake_amdsmi_spec(root, spec).replace("\n", "|") + "|no_libdrm=1"
    outs = {}
    for backend in ("sysfs", "amdsmi"):
        out = tmp_path / f"gfd-{backend}"
        run_daemon(binary, "--oneshot", "--no-timestamp", f"--backend={backend}", f"--sysfs-root={root}",
                   f"--machine-type-file={root}/sys/class/dmi/id/product_name", f"--mig-strategy={c['strategy']}",
                   f"--output-file={out}", env={"GFD_AMDSMI_LIBRARY": str(FAKE), "GFD_FAKE_AMDSMI_SPEC": fake_spec},
                   check=True)
        outs[backend] = out.read_text()
    assert outs["amdsmi"] == outs["sysfs"]
    labels = golden.parse_labels(outs["amdsmi"])
    assert "MI355" in labels["amd.com/gpu.product"]
    assert labels["amd.com/gpu.virtualization-mode"] == "baremetal"


@pytest.mark.skipif(not FAKE.exists(), reason="libfake_amdsmi.so not built")
def test_without_libdrm_or_fru_name_both_backends_use_the_device_model(binary, tmp_path):
    """No marketing name from amd-smi (no libdrm) and no board FRU
    product_name attribute: both backends fall back to the model of the PCI
    device ID, so the product label stays the same."""
    spec = synth.NodeSpec(gpus=[synth.GpuSpec() for _ in range(2)], seed=24)
    root = synth.make_node(tmp_path / "root", spec)
    for f in root.glob("sys/bus/pci/devices/*/product_name"):
        f.unlink()
    # No FRU: the board-info call has nothing to report either.
    fake_spec = (synth.fake_amdsmi_spec(root, spec).replace("\n", "|") +
                 "|no_libdrm=1|fail=amdsmi_get_gpu_board_info:2")
    outs = {}
    for backend in ("sysfs", "amdsmi"):
        out = tmp_path / f"gfd-{backend}"
        run_daemon(binary, "--oneshot", "--no-timestamp", f"--backend={backend}", f"--sysfs-root={root}",
                   f"--machine-type-file={root}/sys/class/dmi/id/product_name", f"--output-file={out}",
                   env={"GFD_AMDSMI_LIBRARY": str(FAKE), "GFD_FAKE_AMDSMI_SPEC": fake_spec}, check=True)
        outs[backend] = out.read_text()
    assert outs["amdsmi"] == outs["sysfs"]
    assert "MI3" in golden.parse_labels(outs["amdsmi"])["amd.com/gpu.product"]


def _loop_files(binary, args, env, cycles_after, marker, timeout=20.0):
    """Run the loop daemon until `marker` is logged and `cycles_after` more
    cycles have written the feature file; return (stderr, the file's
    content after every cycle, in order)."""
    import os
    import signal
    import subprocess
    import time

    out = next(a.split("=", 1)[1] for a in args if a.startswith("--output-file="))
    p = subprocess.Popen([binary, "--sleep-interval=20ms", *args], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                         text=True, env={**{k: v for k, v in os.environ.items() if not k.startswith("GFD_")}, **env})
    err, files, left = [], [], None
    try:
        end = time.monotonic() + timeout
        for line in p.stderr:
            err.append(line)
            if marker in line:
                left = cycles_after
            if "Sleeping for" in line:  # the cycle's file is in place
                with open(out) as f:
                    files.append(f.read())
                if left is not None:
                    left -= 1
                    if left <= 0:
                        break
            if time.monotonic() > end:
                break
    finally:
        p.send_signal(signal.SIGTERM)
        _, rest = p.communicate(timeout=30)
        err.append(rest or "")
    return "".join(err), files


@pytest.mark.skipif(not FAKE.exists(), reason="libfake_amdsmi.so not built")
@pytest.mark.parametrize("agree", [True, False], ids=["agree", "disagree"])
def test_warm_start_switch_never_changes_the_published_labels(binary, tmp_path, agree):
    """The loop daemon labels its first cycles from KFD while amd-smi starts
    in the background (here: 60 ms, so several KFD cycles publish first).
    When amd-smi is ready it takes over if it describes the GPUs as KFD did;
    if it does not, the daemon logs the difference once and keeps labeling
    from KFD until the next restart - the published labels never change
    because a backend finished starting (a CPX node, whose partitions are
    where the two backends could disagree)."""
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(compute_partition="CPX")], seed=31)
    root = synth.make_node(tmp_path / "root", spec)
    fake = synth.fake_amdsmi_spec(root, spec) + "\ninit_latency_us=60000"
    if not agree:
        fake = fake.replace("name=AMD Instinct MI355 OAM", "name=AMD Instinct MI355X")
    env = {"GFD_AMDSMI_LIBRARY": str(FAKE), "GFD_FAKE_AMDSMI_SPEC": fake.replace("\n", "|")}
    err, files = _loop_files(binary, ["--backend=auto", f"--sysfs-root={root}", f"--output-file={tmp_path / 'gfd'}",
                                      f"--machine-type-file={root}/sys/class/dmi/id/product_name", "--mig-strategy=single"],
                             env, cycles_after=5, marker="initialized in the background in")
    assert "initialized in the background in" in err, err[-3000:]
    switched = err.split("initialized in the background in", 1)[0]
    assert switched.count("Writing labels to output file") >= 1, err[-3000:]  # KFD published first
    assert err.count("describes the GPUs differently") == (0 if agree else 1), err[-3000:]
    if agree:
        assert "Using the amdsmi(persistent) manager (initialized in the background" in err
    else:
        assert "labeling from the sysfs manager until the next restart" in err
        assert "Using the amdsmi(persistent) manager" not in err
    # Byte-identical feature files across the switch: not a single change.
    assert len(files) >= 6 and len(set(files)) == 1, [f.splitlines()[:3] for f in files]
    assert golden.parse_labels(files[-1])["amd.com/gpu.count"] == "8"
