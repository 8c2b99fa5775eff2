"""Python-extension tests: the in-process API over the native core
(YAML/config parsing, durations, resource names, sessions over synthetic
trees).  Everything here runs the C++ code in gpu_feature_discovery_amd/_gfd."""

from __future__ import annotations

import pytest

from gpu_feature_discovery_amd.utils import golden, synth


def test_native_module_is_the_in_tree_extension(native):
    import gpu_feature_discovery_amd as gfd

    assert native.__file__.startswith(str(gfd.PACKAGE_DIR))
    assert native.version().startswith("v")


def test_parse_yaml_and_json(native):
    assert native.parse_yaml("a: [1, {b: yes}]\nc: 'x'\n") == {"a": [1, {"b": True}], "c": "x"}
    assert native.parse_yaml('{"a": 1.5, "b": null}') == {"a": 1.5, "b": None}
    with pytest.raises(native.GfdError):
        native.parse_yaml("a: [1\n")


def test_parse_config_roundtrip(native):
    js = native.parse_config("flags:\n  migStrategy: mixed\n  gfd:\n    sleepInterval: 2m\n")
    assert '"migStrategy": "mixed"' in js and '"sleepInterval": "2m0s"' in js
    with pytest.raises(native.GfdError, match="unknown version"):
        native.parse_config("version: v9\n")


@pytest.mark.parametrize("text,ns", [("1h2m3s", 3723 * 10**9), ("250ms", 250 * 10**6), ("0", 0), ("1.5us", 1500)])
def test_durations(native, text, ns):
    assert native.parse_duration(text) == ns


def test_format_duration(native):
    assert native.format_duration(60 * 10**9) == "1m0s"


def test_resource_names(native):
    assert native.new_resource_name("partition-cpx.1xcd.36gb") == "amd.com/partition-cpx.1xcd.36gb"
    with pytest.raises(native.GfdError):
        native.new_resource_name("UPPER")


def test_sanitize_label_value(native):
    assert native.sanitize_label_value("AMD Instinct MI355X") == "AMD-Instinct-MI355X"


def test_session_over_synthetic_tree(native, tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=4, compute_partition="QPX", seed=11)
    s = native.Session(["--backend=sysfs", f"--sysfs-root={root}", "--mig-strategy=mixed", "--no-timestamp",
                        f"--output-file={tmp_path / 'gfd'}"])
    assert s.backend == "sysfs"
    devs = s.devices()
    assert len(devs) == 4 and all(d["partitioned"] for d in devs)
    assert all(len(d["partitions"]) == 4 for d in devs)
    assert devs[0]["partitions"][0]["name"] == "qpx.2xcd.72gb"
    r = s.cycle(True)
    assert (tmp_path / "gfd").read_text() == r["rendered"]
    labels = golden.parse_labels(r["rendered"])
    assert labels["amd.com/partition-qpx.2xcd.72gb.count"] == "16"
    assert labels["amd.com/partition-qpx.2xcd.72gb.compute-units"] == "64"


def test_session_bench_returns_per_step_times(native, tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=2)
    s = native.Session(["--backend=sysfs", f"--sysfs-root={root}", f"--output-file={tmp_path / 'gfd'}"])
    ns = s.bench(25, 5, True)
    assert len(ns) == 25 and all(x > 0 for x in ns)


def test_closing_one_session_keeps_another_sessions_kept_files(native, tmp_path):
    """A loop-mode session keeps the feature file its last write swapped out
    (gfd-tmp/) for the next write; closing another session with a different
    output leaves that file alone, and closing this one removes it."""
    import gc

    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=1)
    outs = [tmp_path / "a" / "gfd", tmp_path / "b" / "gfd"]
    sessions = []
    for out in outs:
        out.parent.mkdir()
        s = native.Session(["--backend=sysfs", f"--sysfs-root={root}", f"--output-file={out}", "--sleep-interval=1s"])
        s.cycle(True)
        s.cycle(True)  # the second write swaps the first file out, into gfd-tmp/
        sessions.append(s)
    kept = [sorted((out.parent / "gfd-tmp").iterdir()) for out in outs]
    assert all(len(k) == 1 for k in kept), kept
    del s
    sessions.pop()  # b's session ends
    gc.collect()
    assert not list((outs[1].parent / "gfd-tmp").iterdir())
    assert sorted((outs[0].parent / "gfd-tmp").iterdir()) == kept[0]  # a's kept file is untouched
    sessions[0].cycle(True)  # and a's next write still reuses it
    assert sorted((outs[0].parent / "gfd-tmp").iterdir()) == kept[0]
    sessions.clear()
    gc.collect()
    assert not list((outs[0].parent / "gfd-tmp").iterdir())


def test_session_env_precedence(native, tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=1)
    s = native.Session([f"--sysfs-root={root}", "--output-file="],
                       env={"GFD_BACKEND": "sysfs", "GFD_MIG_STRATEGY": "single", "GFD_NO_TIMESTAMP": "1"})
    labels = s.cycle(False)["labels"]
    assert labels["amd.com/partition.strategy"] == "single"
    assert "amd.com/gfd.timestamp" not in labels


def test_session_usage_error(native):
    with pytest.raises(native.UsageError, match="flag provided but not defined"):
        native.Session(["--nope"])


def test_session_errors_surface(native, tmp_path):
    s = native.Session(["--backend=sysfs", f"--sysfs-root={tmp_path}", "--output-file="])
    with pytest.raises(native.GfdError, match="KFD topology not available"):
        s.cycle(False)


@pytest.mark.parametrize("kind", ["spx8", "sriov-host", "sriov-host-privileged", "guest-vf", "guest-vf-unbound",
                                  "host-vfio-pf", "guest-vf-one-unprobed", "host-unbound-gpu"])
def test_bound_sriov_source_matches_the_whole_bus(native, tmp_path, kind):
    """The daemon's SR-IOV source (the functions amdgpu / gim bind, plus
    their VFs) hands the labeler the same functions, field for field, as the
    reference-style scan of the whole PCI bus - on nodes of every SR-IOV
    shape (sriov/bound.h).  A guest whose amdgpu is not loaded has nothing
    bound: the daemon then falls back to the bus scan, which this source on
    its own reports as nothing."""
    gim = None
    if kind == "spx8":
        gpus = [synth.GpuSpec() for _ in range(8)]
    elif kind.startswith("sriov-host"):
        gpus = [synth.GpuSpec(sriov={"total": 8, "num": 3, "vf_device": 0x75B3}), synth.GpuSpec()]
        gim = "8.1.0.K"
    elif kind == "host-vfio-pf":
        # A PF handed to vfio-pci, its VFs enabled, next to an amdgpu GPU.
        gpus = [synth.GpuSpec(sriov={"total": 8, "num": 2, "vf_device": 0x75B3}, driver="vfio-pci", kfd=False),
                synth.GpuSpec()]
    elif kind == "guest-vf-one-unprobed":
        # A VM with two VFs; amdgpu failed to probe the second.
        gpus = [synth.GpuSpec(vf=True), synth.GpuSpec(vf=True, driver=None, kfd=False)]
    elif kind == "host-unbound-gpu":
        # Bare metal: a GPU no driver binds, next to an amdgpu one.
        gpus = [synth.GpuSpec(), synth.GpuSpec(driver=None, kfd=False)]
    else:
        gpus = [synth.GpuSpec(vf=True, driver=None if kind.endswith("unbound") else "auto")]
    guest = kind.startswith("guest")
    root = synth.make_node(tmp_path / "node", synth.NodeSpec(gpus=gpus, gim_version=gim, seed=11, hypervisor=guest,
                                                              privileged=kind.endswith("privileged")))
    bound = native.pci_functions(str(root), "bound")
    bus = native.pci_functions(str(root), "bus")
    daemon = native.pci_functions(str(root), "daemon")
    # The daemon's labels are the bus scan's on every node shape.
    assert native.sriov_labels(str(root), "daemon") == native.sriov_labels(str(root), "bus")
    if kind == "host-unbound-gpu":
        # On a host the daemon does not read the bus: the unbound GPU (no VFs,
        # so no SR-IOV state) is not among its functions, and the labeler
        # classifies it as nothing either way.
        assert len(bus) == 2 and len(bound) == len(daemon) == 1
        assert native.sriov_labels(str(root), "daemon") == {}
        return
    # Everywhere else, function for function (a VM reads its bus too).
    assert daemon == bus
    if kind == "guest-vf-unbound":
        assert bound == [] and len(bus) == 1
        return
    if kind == "guest-vf-one-unprobed":
        assert len(bound) == 1 and len(bus) == 2
        return
    assert bound == bus
    assert len(bound) == {"spx8": 8, "guest-vf": 1, "host-vfio-pf": 4}.get(kind, 2 + 3)
