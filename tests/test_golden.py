"""End-to-end golden tests of the daemon binary.

BASELINE.json config 1 ("mock/null resource manager on CPU,
mig-strategy=none, golden-file diff vs tests/expected-output.txt") plus the
partition-strategy and SR-IOV goldens.  Mirrors the reference's
cmd/gpu-feature-discovery/main_test.go (TestRunOneshot, TestRunWithNoTimestamp)
and mig_test.go (TestMigStrategy{None,Single,Mixed,...}), but:

* byte goldens (tests/golden/*.txt) pin the exact, sorted feature file;
* regex goldens (tests/expected-output*.txt) are checked bidirectionally.

Regenerate byte goldens with GFD_UPDATE_GOLDENS=1 (then review the diff).
"""

from __future__ import annotations

import os
from pathlib import Path

import pytest

from conftest import FIXTURES, GOLDEN, TESTS, run_daemon
from gpu_feature_discovery_amd.utils import golden, synth

UPDATE = os.environ.get("GFD_UPDATE_GOLDENS") == "1"


def _oneshot(binary, tmp_path, *args, timestamp=False, sysfs_root=None, machine=None):
    out = tmp_path / "gfd"
    root = sysfs_root or str(synth.make_node(tmp_path / "empty-root", synth.NodeSpec(gpus=[])))
    mt = machine or str(Path(root) / "sys/class/dmi/id/product_name")
    argv = ["--oneshot", f"--output-file={out}", f"--machine-type-file={mt}", f"--sysfs-root={root}", *args]
    if not timestamp:
        argv.append("--no-timestamp")
    run_daemon(binary, *argv, check=True)
    text = out.read_text()
    golden.parse_labels(text)  # no duplicates, key=value lines
    return text


def _mock(name):
    return ["--backend=mock", f"--mock-file={FIXTURES / name}"]


# ---- BASELINE config 1: mock backend, strategy none -------------------------

def test_config1_mock_none_byte_golden(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("full-gpu.yaml"), "--mig-strategy=none")
    golden.check_byte_golden(text, GOLDEN / "mock-none.txt", UPDATE)


def test_config1_mock_none_regex_golden(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("full-gpu.yaml"), timestamp=True)
    golden.check_regex_golden(text, TESTS / "expected-output.txt", select=lambda ln: "sriov" not in ln)
    labels = golden.parse_labels(text)
    assert labels["amd.com/gpu.count"] == "1"
    assert labels["amd.com/gpu.product"] == "MOCKMODEL"
    assert labels["amd.com/gpu.memory"] == "300"


def test_no_timestamp_omits_label(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("full-gpu.yaml"))
    assert "amd.com/gfd.timestamp=" not in text


def test_null_backend_writes_only_timestamp(binary, tmp_path):
    text = _oneshot(binary, tmp_path, "--backend=null", timestamp=True)
    assert list(golden.parse_labels(text)) == ["amd.com/gfd.timestamp"]


# ---- Partition strategies (mig_test.go analogues) ----------------------------

def test_strategy_none_with_partitioned_gpu(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("partitioned-single.yaml"), "--mig-strategy=none")
    labels = golden.parse_labels(text)
    assert labels["amd.com/gpu.count"] == "1"
    assert labels["amd.com/gpu.product"] == "MOCKMODEL"
    assert labels["amd.com/gpu.memory"] == "300"
    assert labels["amd.com/gpu.replicas"] == "0"
    assert "amd.com/partition.strategy" not in labels


def test_strategy_single_no_partitioned_devices(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("full-gpu.yaml"), "--mig-strategy=single")
    labels = golden.parse_labels(text)
    assert labels["amd.com/partition.strategy"] == "single"
    assert labels["amd.com/gpu.count"] == "1"
    assert labels["amd.com/gpu.product"] == "MOCKMODEL"
    assert labels["amd.com/gpu.memory"] == "300"


def test_strategy_single(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("partitioned-single.yaml"), "--mig-strategy=single", timestamp=True)
    golden.check_regex_golden(text, TESTS / "expected-output-partition-single.txt")
    labels = golden.parse_labels(text)
    assert labels["amd.com/gpu.count"] == "2"
    assert labels["amd.com/gpu.product"] == "MOCKMODEL-PARTITION-cpx.1xcd.20gb"
    assert labels["amd.com/gpu.memory"] == "20"
    golden.check_byte_golden(_oneshot(binary, tmp_path, *_mock("partitioned-single.yaml"), "--mig-strategy=single"),
                             GOLDEN / "mock-single.txt", UPDATE)


def test_strategy_single_invalid_when_empty(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("partitioned-empty.yaml"), "--mig-strategy=single")
    labels = golden.parse_labels(text)
    assert labels["amd.com/gpu.product"] == "MOCKMODEL-PARTITION-INVALID"
    assert labels["amd.com/gpu.count"] == "0"
    assert labels["amd.com/gpu.replicas"] == "0"
    assert labels["amd.com/gpu.memory"] == "0"


def test_strategy_single_invalid_with_mixed_profiles(binary, tmp_path):
    labels = golden.parse_labels(_oneshot(binary, tmp_path, *_mock("partitioned-mixed.yaml"), "--mig-strategy=single"))
    assert labels["amd.com/gpu.product"] == "MOCKMODEL-PARTITION-INVALID"


def test_strategy_mixed(binary, tmp_path):
    text = _oneshot(binary, tmp_path, *_mock("partitioned-mixed.yaml"), "--mig-strategy=mixed", timestamp=True)
    golden.check_regex_golden(text, TESTS / "expected-output-partition-mixed.txt")
    labels = golden.parse_labels(text)
    assert labels["amd.com/partition.strategy"] == "mixed"
    assert labels["amd.com/gpu.count"] == "1"
    assert labels["amd.com/gpu.product"] == "MOCKMODEL"
    assert labels["amd.com/gpu.memory"] == "300"
    assert labels["amd.com/partition-cpx.1xcd.20gb.count"] == "1"
    assert labels["amd.com/partition-qpx.2xcd.5gb.count"] == "1"
    golden.check_byte_golden(_oneshot(binary, tmp_path, *_mock("partitioned-mixed.yaml"), "--mig-strategy=mixed"),
                             GOLDEN / "mock-mixed.txt", UPDATE)


def test_unknown_strategy_fails_with_devices(binary, tmp_path):
    cp = run_daemon(binary, "--oneshot", "-o", str(tmp_path / "x"), *_mock("full-gpu.yaml"), "--mig-strategy=bogus",
                    f"--sysfs-root={tmp_path}")
    assert cp.returncode == 1
    assert "unknown strategy: bogus" in cp.stderr


# ---- Synthetic MI355X nodes (sysfs backend) ----------------------------------

@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_synthetic_spx_node(binary, tmp_path, n):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=n, seed=n)
    text = _oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root))
    golden.check_byte_golden(text.replace(f"amd.com/gpu.count={n}\n", "amd.com/gpu.count=N\n"),
                             GOLDEN / "synthetic-spx.txt", UPDATE)
    assert golden.parse_labels(text)["amd.com/gpu.count"] == str(n)


def test_synthetic_spx_matches_regex_golden(binary, tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=8, seed=3)
    text = _oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root), timestamp=True)
    golden.check_regex_golden(text, TESTS / "expected-output.txt")


# Partition layouts: current kernels report partition k of a GPU at bb:00.0
# as bb:00.k in its KFD location_id (kfd_topology.c ORs the XCP node id in);
# older ones give every partition the parent's location.  Both must produce
# the same labels (resource/physical.h).
LAYOUTS = ["function", "shared", "distinct-ids"]


@pytest.mark.parametrize("layout", LAYOUTS)
def test_synthetic_cpx_single(binary, tmp_path, layout):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=8, compute_partition="CPX", seed=5,
                                  partition_layout=layout)
    text = _oneshot(binary, tmp_path, "--backend=sysfs", "--mig-strategy=single", sysfs_root=str(root))
    golden.check_byte_golden(text, GOLDEN / "synthetic-cpx-single.txt", UPDATE)
    labels = golden.parse_labels(text)
    assert labels["amd.com/gpu.count"] == "64"
    assert labels["amd.com/gpu.product"] == "AMD-Instinct-MI355-OAM-PARTITION-cpx.1xcd.36gb"
    assert labels["amd.com/gpu.compute-units"] == "32"


@pytest.mark.parametrize("layout", LAYOUTS)
def test_synthetic_dpx_nps2_mixed(binary, tmp_path, layout):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=4, compute_partition="DPX", memory_partition="NPS2",
                                  seed=6, partition_layout=layout)
    text = _oneshot(binary, tmp_path, "--backend=sysfs", "--mig-strategy=mixed", sysfs_root=str(root))
    golden.check_byte_golden(text, GOLDEN / "synthetic-dpx-nps2-mixed.txt", UPDATE)
    labels = golden.parse_labels(text)
    assert labels["amd.com/partition-dpx.4xcd.144gb.count"] == "8"
    assert labels["amd.com/partition-dpx.4xcd.144gb.memory-partition"] == "NPS2"


@pytest.mark.parametrize("layout", LAYOUTS)
def test_two_gpu_cpx_single_and_mixed(binary, tmp_path, layout):
    """Round-1 review reproduction: 2 GPUs in CPX, partition addresses with
    the index in the function bits, must count 16 partitions, not 16 GPUs."""
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=2, compute_partition="CPX", seed=11,
                                  partition_layout=layout)
    single = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", "--mig-strategy=single",
                                          sysfs_root=str(root)))
    assert single["amd.com/gpu.count"] == "16"
    assert single["amd.com/gpu.product"] == "AMD-Instinct-MI355-OAM-PARTITION-cpx.1xcd.36gb"
    assert single["amd.com/gpu.compute-partition"] == "CPX"
    assert single["amd.com/gpu.xgmi.links"] == "7"
    mixed = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", "--mig-strategy=mixed",
                                         sysfs_root=str(root)))
    assert mixed["amd.com/partition-cpx.1xcd.36gb.count"] == "16"
    assert mixed["amd.com/gpu.count"] == "2"
    assert mixed["amd.com/gpu.memory"] == str(synth.MI355X_VRAM_BYTES >> 20)
    assert mixed["amd.com/gpu.compute-partition"] == "CPX"


@pytest.mark.parametrize("layout", LAYOUTS)
def test_one_visible_cpx_partition(binary, tmp_path, layout):
    """A pod allocated one CPX partition: its KFD node reports bb:00.3 (not a
    PCI function); the GPU-wide attributes come from bb:00.0."""
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(compute_partition="CPX", visible_partitions=[3])],
                          partition_layout=layout, seed=12)
    root = str(synth.make_node(tmp_path / "root", spec))
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", "--mig-strategy=single",
                                          sysfs_root=root))
    assert labels["amd.com/gpu.count"] == "1"
    assert labels["amd.com/gpu.product"] == "AMD-Instinct-MI355-OAM-PARTITION-cpx.1xcd.36gb"
    assert labels["amd.com/gpu.compute-partition"] == "CPX"
    assert labels["amd.com/gpu.memory-partition"] == "NPS1"
    assert labels["amd.com/gpu.partition.capable"] == "true"


def test_partitions_of_other_families_keep_exact_addresses(binary, tmp_path):
    """Function-bit masking applies to partition-capable families (gfx94x,
    gfx950) only: two gfx90a GPUs that are functions of one slot stay two GPUs."""
    gpus = [synth.GpuSpec(gfx_target_version=90010, product_name="AMD Instinct MI250X", cus=104, xcds=1)
            for _ in range(2)]
    root = synth.make_node(tmp_path / "root", synth.NodeSpec(gpus=gpus, seed=13))
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    # Move the second GPU onto function 1 of the first GPU's slot.
    props = [kfd / d / "properties" for d in sorted(os.listdir(kfd), key=int)]
    gpu_props = [p for p in props if "simd_count 0\n" not in p.read_text()]
    first_loc = int(next(ln.split()[1] for ln in gpu_props[0].read_text().splitlines() if ln.startswith("location_id")))
    text = gpu_props[1].read_text()
    old_loc = next(ln for ln in text.splitlines() if ln.startswith("location_id"))
    text = text.replace(old_loc, f"location_id {first_loc | 1}")
    # ... and with the same (e.g. unreported) unique_id, so only the address tells them apart.
    first_uid = next(ln for ln in gpu_props[0].read_text().splitlines() if ln.startswith("unique_id"))
    old_uid = next(ln for ln in text.splitlines() if ln.startswith("unique_id"))
    gpu_props[1].write_text(text.replace(old_uid, first_uid))
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root)))
    assert labels["amd.com/gpu.count"] == "2"


def test_synthetic_sriov_pf(binary, tmp_path):
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(sriov={"total": 8, "num": 4, "vf_device": 0x75B3})], seed=7)
    root = synth.make_node(tmp_path / "root", spec)
    text = _oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root))
    golden.check_regex_golden(text, TESTS / "expected-output-sriov.txt", select=lambda ln: "sriov" in ln)
    labels = golden.parse_labels(text)
    assert labels["amd.com/sriov.present"] == "true"
    # Per-function order: the PF then its VFs; the last function wins.
    assert labels["amd.com/sriov.role"] in ("pf", "vf")
    assert labels["amd.com/sriov.num-vfs"] == "4"
    assert labels["amd.com/sriov.total-vfs"] == "8"
    golden.check_byte_golden(text, GOLDEN / "synthetic-sriov.txt", UPDATE)


def test_sriov_host_driver_version_on_gim_host(binary, tmp_path):
    """vgpu.go:44-52 labels the host driver version; on an MxGPU host that is
    the GIM module's version.  A guest cannot see it (no host-driver record
    in the VF's config space): the label is absent there."""
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(sriov={"total": 8, "num": 4})], gim_version="8.1.0.K", seed=7)
    root = synth.make_node(tmp_path / "root", spec)
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root)))
    assert labels["amd.com/sriov.role"] == "pf"
    assert labels["amd.com/sriov.host-driver-version"] == "8.1.0.K"
    guest = synth.NodeSpec(gpus=[synth.GpuSpec(vf=True)], hypervisor=True, gim_version="8.1.0.K", seed=9)
    root = synth.make_node(tmp_path / "guest", guest)
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root)))
    assert labels["amd.com/sriov.role"] == "vf"
    assert "amd.com/sriov.host-driver-version" not in labels


def test_synthetic_sriov_privileged_config_space(binary, tmp_path):
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(sriov={"total": 8, "num": 2})], privileged=True, seed=8)
    root = synth.make_node(tmp_path / "root", spec)
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root)))
    assert labels["amd.com/sriov.num-vfs"] == "2"


def test_amdsmi_and_sysfs_label_sets_are_identical_in_shape(binary, tmp_path):
    """The regex golden used for hardware runs is the same file the synthetic
    tree satisfies, so both backends must emit the same 22 keys."""
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=1)
    keys = set(golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root), timestamp=True)))
    assert len(keys) == len(golden.load_regexes(TESTS / "expected-output.txt"))


def test_synthetic_sriov_vf_nps4_mixed(binary, tmp_path):
    """BASELINE config 5: an MxGPU guest - SR-IOV virtual functions in
    QPX/NPS4 - under the mixed strategy (the reference's vGPU + MIG-mixed
    analogue)."""
    spec = synth.NodeSpec(gpus=[synth.GpuSpec(vf=True, compute_partition="QPX", memory_partition="NPS4")
                                for _ in range(2)], hypervisor=True, seed=9)
    root = synth.make_node(tmp_path / "root", spec)
    text = _oneshot(binary, tmp_path, "--backend=sysfs", "--mig-strategy=mixed", sysfs_root=str(root))
    golden.check_byte_golden(text, GOLDEN / "synthetic-sriov-vf-nps4-mixed.txt", UPDATE)
    # A guest VF has no VFs of its own: present + role only.
    golden.check_regex_golden(text, TESTS / "expected-output-sriov-vf.txt", select=lambda ln: "sriov" in ln)
    labels = golden.parse_labels(text)
    assert labels["amd.com/sriov.role"] == "vf"
    assert labels["amd.com/gpu.virtualization-mode"] == "guest"
    assert labels["amd.com/gpu.memory-partition"] == "NPS4"
    assert labels["amd.com/partition-qpx.2xcd.72gb.count"] == "8"
    assert labels["amd.com/partition-qpx.2xcd.72gb.memory-partition"] == "NPS4"


def test_synthetic_passthrough_vm(binary, tmp_path):
    """A whole GPU passed through to a VM: hypervisor CPU flag, no SR-IOV."""
    root = synth.make_node(tmp_path / "root", synth.NodeSpec(gpus=[synth.GpuSpec()], hypervisor=True, seed=10))
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", sysfs_root=str(root)))
    assert labels["amd.com/gpu.virtualization-mode"] == "passthrough"
    assert not any("sriov" in k for k in labels)


# ---- Node-true ROCm version (--host-root / --rocm-version-file) --------------

def _host(tmp_path, version: str | None, link: str = "/opt/rocm-{v}"):
    host = tmp_path / "host"
    (host / "opt").mkdir(parents=True)
    if version:
        d = host / f"opt/rocm-{version}/.info"
        d.mkdir(parents=True)
        (d / "version").write_text(version + "-57\n")
        (host / "opt/rocm").symlink_to(link.format(v=version))
    return host


def test_host_root_labels_the_nodes_rocm_not_the_images(binary, tmp_path):
    """The pod's own tree says 7.2 (what an image would carry); the host's
    /opt/rocm -> /opt/rocm-6.4.1 (an absolute link, re-rooted under the mount)
    says 6.4: the labels describe the node."""
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=1, rocm_version="7.2.0")
    host = _host(tmp_path, "6.4.1")
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", f"--host-root={host}",
                                          sysfs_root=str(root)))
    assert (labels["amd.com/rocm.runtime.major"], labels["amd.com/rocm.runtime.minor"]) == ("6", "4")


def test_driver_only_host_gets_no_runtime_labels(binary, tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=1, rocm_version="7.2.0")
    host = _host(tmp_path, None)
    out = tmp_path / "gfd"
    cp = run_daemon_checked(binary, tmp_path, root, f"--host-root={host}", out=out)
    labels = golden.parse_labels(out.read_text())
    assert "amd.com/rocm.runtime.major" not in labels
    assert labels["amd.com/driver.major"] == "6"
    assert "no ROCm release found on the node" in cp.stderr


def test_host_root_without_opt_mount_fails_loudly(binary, tmp_path):
    """A manifest that sets GFD_HOST_ROOT but does not mount the host's /opt
    there: the cycle fails with the reason instead of dropping the
    amd.com/rocm.runtime.* labels with a warning."""
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=1, rocm_version="7.2.0")
    host = tmp_path / "host"
    host.mkdir()
    cp = run_daemon(binary, "--oneshot", "--backend=sysfs", f"--sysfs-root={root}", "--output-file=",
                    f"--host-root={host}")
    assert cp.returncode == 1
    assert "has no opt/ directory" in cp.stderr


def test_explicit_rocm_version_file(binary, tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=1, rocm_version="7.2.0")
    f = tmp_path / "version"
    f.write_text("6.3.3\n")
    labels = golden.parse_labels(_oneshot(binary, tmp_path, "--backend=sysfs", f"--rocm-version-file={f}",
                                          sysfs_root=str(root)))
    assert labels["amd.com/rocm.runtime.minor"] == "3"
    cp = run_daemon(binary, "--oneshot", "--backend=sysfs", f"--sysfs-root={root}", "--output-file=",
                    f"--rocm-version-file={tmp_path / 'missing'}")
    assert cp.returncode == 1
    assert "unable to read the ROCm version file" in cp.stderr


def run_daemon_checked(binary, tmp_path, root, *args, out):
    return run_daemon(binary, "--oneshot", "--no-timestamp", "--backend=sysfs", f"--sysfs-root={root}",
                      f"--machine-type-file={root}/sys/class/dmi/id/product_name", f"--output-file={out}", *args,
                      check=True)


@pytest.mark.parametrize("golden_file", sorted(p.name for p in (TESTS / "golden").glob("*.txt")))
def test_goldens_are_valid_kubernetes_labels(golden_file):
    """Every label of every byte golden passes the syntax checks NFD and the
    API server apply (a rejected label is silently missing from the Node)."""
    labels = golden.parse_labels((TESTS / "golden" / golden_file).read_text())
    assert labels and golden.k8s_label_problems(labels) == []


def test_label_syntax_check_rejects_bad_labels():
    bad = {"amd.com/gpu.product": "-x", "amd.com/" + "n" * 64: "1", "AMD.com/x": "1", "a/b/c": "1",
           "amd.com/ok": "v" * 64}
    flagged = {p.split(":")[0].split("=")[0] for p in golden.k8s_label_problems(bad)}
    assert flagged == set(bad)
    assert golden.k8s_label_problems({"amd.com/partition-cpx.1xcd.36gb.count": "16", "amd.com/x": ""}) == []
