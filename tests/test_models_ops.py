"""The Python device model and the in-process ops API.

* ``models.mi355x`` predicts partition geometry and profile names; the
  native daemon must agree for every (compute, memory) mode combination
  (synthetic trees, mixed strategy).
* ``ops.Labeler`` drives the native core in-process (mock and synthetic
  backends here; the GPU suite and bench.py use it on hardware).
"""

from __future__ import annotations

import pytest

from conftest import FIXTURES, TESTS
from gpu_feature_discovery_amd.models import mi355x
from gpu_feature_discovery_amd.ops import CycleResult, Labeler, devices, label_once
from gpu_feature_discovery_amd.utils import golden, synth


def test_model_constants_match_measured_hardware():
    assert mi355x.VRAM_MIB == 294896
    assert mi355x.CUS == mi355x.XCDS * 32
    assert mi355x.partition_profile("CPX", 1, 36862) == "cpx.1xcd.36gb"
    assert mi355x.partition_profile("", 8, 294896) == "xcp.8xcd.288gb"


def test_partition_geometry_conserves_the_gpu():
    for c, m in mi355x.valid_modes():
        parts = mi355x.partitions(c, m)
        assert len(parts) == mi355x.PARTITIONS_PER_MODE[c]
        assert sum(p.xcds for p in parts) == mi355x.XCDS
        assert sum(p.compute_units for p in parts) == mi355x.CUS
        assert sum(p.memory_mib for p in parts) <= mi355x.VRAM_MIB
    with pytest.raises(ValueError):
        mi355x.partitions("SPX", "NPS4")


@pytest.mark.parametrize("compute,memory", [(c, m) for c, m in mi355x.valid_modes() if c != "SPX"])
def test_daemon_profile_names_match_model(tmp_path, compute, memory):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=2, compute_partition=compute, memory_partition=memory)
    labels = label_once(["--backend=sysfs", f"--sysfs-root={root}", "--mig-strategy=mixed", "--output-file=",
                         f"--machine-type-file={root}/sys/class/dmi/id/product_name"]).labels
    (part,) = {p.profile for p in mi355x.partitions(compute, memory)}
    n = 2 * mi355x.PARTITIONS_PER_MODE[compute]
    assert labels[f"amd.com/partition-{part}.count"] == str(n), sorted(labels)
    assert labels[f"amd.com/partition-{part}.memory-partition"] == memory


def test_labeler_on_mock_fixture(tmp_path):
    out = tmp_path / "gfd"
    lab = Labeler(["--backend=mock", f"--mock-file={FIXTURES / 'full-gpu.yaml'}", f"--output-file={out}",
                   "--no-timestamp"])
    assert lab.backend
    r = lab.cycle(write=True)
    assert isinstance(r, CycleResult)
    assert r.labels["amd.com/gpu.product"] == "MOCKMODEL"
    assert out.read_text() == r.rendered
    assert r.total_ms > 0 and any(name == "write" for name, _ in r.phases_ms)
    ms = lab.bench(5, 1, write=False)
    assert len(ms) == 5 and all(x > 0 for x in ms)
    assert '"migStrategy"' in lab.config_json


def test_devices_and_label_once_on_synthetic_tree(tmp_path):
    root = synth.make_mi355x_node(tmp_path / "root", n_gpus=4, seed=11)
    args = ["--backend=sysfs", f"--sysfs-root={root}", "--output-file=",
            f"--machine-type-file={root}/sys/class/dmi/id/product_name"]
    devs = devices(args)
    assert len(devs) == 4 and all(d["gfx"] == mi355x.GFX_TARGET for d in devs)
    assert all(d["memory_mib"] == mi355x.VRAM_MIB for d in devs)
    labels = label_once(args).labels
    golden.check_regex_golden("".join(f"{k}={v}\n" for k, v in sorted(labels.items())),
                              TESTS / "expected-output.txt")
