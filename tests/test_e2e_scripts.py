"""The counterparts of the reference's container integration test
(tests/integration-tests.py) and cluster e2e test (tests/e2e-tests.py) -
tests/e2e/integration_docker.py and tests/e2e/e2e_kubectl.py - run as they
are, against a fake `docker` and a fake one-node `kubectl`
(tests/e2e/fakes/): the labeler starts from the manifests' own argv, env
and mounts, and the fake cluster publishes labels the way NFD would (its PCI
source under the worker's class whitelist, its local source only in the
master's -extra-label-ns namespaces).  On CPU the node is a synthetic
MI355X tree; tests/test_gpu.py runs the same on the real MI355X.
"""

from __future__ import annotations

import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

from conftest import REPO
from gpu_feature_discovery_amd.utils import synth

FAKES = REPO / "tests" / "e2e" / "fakes"


def e2e_env(tmp_path, sysfs_root=None, host_opt=None) -> dict:
    env = {k: v for k, v in os.environ.items() if not k.startswith(("GFD_", "FAKE_"))}
    env["PATH"] = f"{FAKES}:{env['PATH']}"
    env["FAKE_RUNTIME_STATE"] = str(tmp_path / "runtime")
    if sysfs_root:
        env["FAKE_SYSFS_ROOT"] = str(sysfs_root)
    if host_opt:
        env["FAKE_HOST_OPT"] = str(host_opt)
    return env


def stop_all(env):
    """Stop whatever the fakes started (the e2e script leaves its DaemonSet)."""
    sys.path.insert(0, str(FAKES))
    os.environ["FAKE_RUNTIME_STATE"] = env["FAKE_RUNTIME_STATE"]
    try:
        import importlib

        rt = importlib.reload(importlib.import_module("_runtime"))
        for pid_file in rt.STATE.glob("*/pid"):
            rt.stop(pid_file.parent.name)
    finally:
        os.environ.pop("FAKE_RUNTIME_STATE", None)
        sys.path.remove(str(FAKES))


def image_libraries(env) -> tuple[list[str], list[str]]:
    """Shared objects the fakes' labeler containers loaded (from the loader
    traces the fake runtime keeps), and those not from the image."""
    sys.path.insert(0, str(FAKES))
    try:
        import _image
    finally:
        sys.path.remove(str(FAKES))
    root = _image.build()
    loaded, foreign = [], []
    for c in Path(env["FAKE_RUNTIME_STATE"]).glob("*/"):
        loaded += _image.loaded_objects(c / "ld")
        foreign += _image.foreign_libraries(root, c / "ld")
    return loaded, foreign


def assert_ran_from_the_image(env):
    loaded, foreign = image_libraries(env)
    assert loaded and not foreign, (loaded, foreign)


def run_integration(env, strategy="none", timeout=60):
    return subprocess.run([sys.executable, str(REPO / "tests/e2e/integration_docker.py"), "gfd-amd:test",
                           f"--strategy={strategy}", "--timeout=30"], capture_output=True, text=True, env=env,
                          timeout=timeout)


def run_e2e(env, strategy=None, timeout=90):
    extra = [f"--strategy={strategy}"] if strategy else []
    return subprocess.run([sys.executable, str(REPO / "tests/e2e/e2e_kubectl.py"), "--timeout=40", *extra],
                          capture_output=True, text=True, env=env, timeout=timeout)


@pytest.fixture()
def node(tmp_path):
    return synth.make_mi355x_node(tmp_path / "node", n_gpus=2, seed=50)


# The node kinds of BASELINE.json's configs that the scripts must handle:
# unpartitioned (SPX/NPS1), every GPU in CPX (the `single` analogue) and
# DPX over NPS2 memory (the `mixed` analogue); with the GPU count each
# kind's `amd.com/gpu.count` has under the `none` strategy.
NODE_KINDS = {
    "spx": dict(compute_partition="SPX", memory_partition="NPS1"),
    "cpx": dict(compute_partition="CPX", memory_partition="NPS1"),
    "dpx-nps2": dict(compute_partition="DPX", memory_partition="NPS2"),
}


def make_kind(tmp_path, kind):
    return synth.make_mi355x_node(tmp_path / f"node-{kind}", n_gpus=2, seed=50, **NODE_KINDS[kind])


@pytest.mark.parametrize("kind", list(NODE_KINDS))
@pytest.mark.parametrize("strategy", ["none", "single", "mixed"])
def test_integration_script_against_fake_docker(tmp_path, kind, strategy):
    node = make_kind(tmp_path, kind)
    env = e2e_env(tmp_path, node, node / "opt")
    try:
        cp = run_integration(env, strategy)
    finally:
        stop_all(env)
    assert cp.returncode == 0, cp.stdout + cp.stderr
    assert "integration test passed" in cp.stdout
    assert "amd.com/rocm.runtime.major=7" in cp.stdout
    labels = dict(ln.split("=", 1) for ln in cp.stdout.splitlines() if ln.startswith("amd.com/"))
    partition = NODE_KINDS[kind]["compute_partition"]
    assert labels["amd.com/gpu.compute-partition"] == partition
    if kind == "cpx" and strategy == "single":
        # The branch the round-3 verdict found broken: the node golden.
        assert labels["amd.com/gpu.product"].endswith("-PARTITION-cpx.1xcd.36gb"), labels
        assert labels["amd.com/gpu.count"] == "16" and labels["amd.com/gpu.arch"] == "gfx950", labels
    if kind == "dpx-nps2" and strategy == "mixed":
        assert labels["amd.com/partition-dpx.4xcd.144gb.count"] == "4", labels
    assert_ran_from_the_image(env)


@pytest.mark.parametrize("kind", list(NODE_KINDS))
@pytest.mark.parametrize("strategy", ["none", "single", "mixed"])
def test_e2e_script_against_fake_cluster(tmp_path, kind, strategy):
    node = make_kind(tmp_path, kind)
    env = e2e_env(tmp_path, node, node / "opt")
    try:
        cp = run_e2e(env, strategy)
    finally:
        stop_all(env)
    assert cp.returncode == 0, cp.stdout + cp.stderr
    assert "e2e test passed" in cp.stdout
    assert f'"amd.com/partition.strategy": "{strategy}"' in cp.stdout or strategy == "none"
    if strategy == "none" or kind == "spx":
        assert '"amd.com/gpu.count": "2"' in cp.stdout
    assert_ran_from_the_image(env)


def test_fake_cluster_enforces_nfd_wiring(tmp_path, node):
    """The fake cluster is strict where a real one is: without amd.com in
    nfd-master's -extra-label-ns no amd.com label is published, and without
    PCI class 12 in the worker's whitelist the labeler's node affinity never
    matches an MI355X node."""
    env = e2e_env(tmp_path, node, node / "opt")
    nfd = (REPO / "deployments/static/nfd.yaml").read_text()
    ds = REPO / "deployments/static/gpu-feature-discovery-daemonset.yaml"
    kubectl = [str(FAKES / "kubectl")]

    def labels():
        import json

        out = subprocess.run(kubectl + ["get", "nodes", "-o", "json"], capture_output=True, text=True, env=env,
                             check=True).stdout
        return json.loads(out)["items"][0]["metadata"]["labels"]

    try:
        bad = tmp_path / "nfd-no-ns.yaml"
        bad.write_text(re.sub(r'^\s*- "-extra-label-ns=amd.com"\n', "", nfd, flags=re.M))
        subprocess.run(kubectl + ["apply", "-f", str(bad)], check=True, env=env, capture_output=True)
        subprocess.run(kubectl + ["apply", "-f", str(ds)], check=True, env=env, capture_output=True)
        import time

        time.sleep(1.0)
        got = labels()
        assert got.get("feature.node.kubernetes.io/pci-1002.present") == "true"
        assert not any(k.startswith("amd.com/") for k in got), got
    finally:
        stop_all(env)
    env2 = e2e_env(tmp_path / "b", node, node / "opt")
    try:
        bad = tmp_path / "nfd-no-class.yaml"
        bad.write_text(nfd.replace('"12", "1200"', '"0b40"'))
        subprocess.run(kubectl + ["apply", "-f", str(bad)], check=True, env=env2, capture_output=True)
        cp = subprocess.run(kubectl + ["apply", "-f", str(ds)], env=env2, capture_output=True, text=True)
        assert "no node matches its affinity" in cp.stderr
    finally:
        stop_all(env2)


def helm_install(env, tmp_path, values=None):
    """`helm install` of the chart's rendering (tests/helm_lite.py) into the
    fake cluster: every rendered document applied with the fake kubectl."""
    import helm_lite
    import yaml

    docs = helm_lite.documents(helm_lite.render_chart(REPO / "deployments/helm/gpu-feature-discovery-amd", values))
    # NFD first, as the e2e script applies it (the labeler's affinity needs
    # the node's PCI labels).
    docs.sort(key=lambda d: 0 if "nfd" in d["metadata"]["name"] else 1)
    manifest = tmp_path / "rendered.yaml"
    manifest.write_text(yaml.safe_dump_all(docs))
    return subprocess.run([str(FAKES / "kubectl"), "apply", "-f", str(manifest)], capture_output=True, text=True,
                          env=env, timeout=60)


def wait_for_node_labels(env, timeout=30.0) -> dict:
    import json
    import time

    end = time.monotonic() + timeout
    labels = {}
    while time.monotonic() < end:
        out = subprocess.run([str(FAKES / "kubectl"), "get", "nodes", "-o", "json"], capture_output=True, text=True,
                             env=env, check=True).stdout
        labels = json.loads(out)["items"][0]["metadata"]["labels"]
        if "amd.com/gfd.timestamp" in labels:
            break
        time.sleep(0.2)
    return labels


def test_helm_chart_installs_into_the_fake_cluster(tmp_path, node):
    """The chart's defaults, rendered and applied: its NFD subchart's worker
    reaches the master Service it names, the node gets its PCI vendor label,
    the labeler DaemonSet schedules on it, and NFD publishes the amd.com
    labels the labeler writes."""
    env = e2e_env(tmp_path, node, node / "opt")
    try:
        cp = helm_install(env, tmp_path)
        assert cp.returncode == 0, cp.stderr
        labels = wait_for_node_labels(env)
    finally:
        stop_all(env)
    assert labels.get("feature.node.kubernetes.io/pci-1002.present") == "true", labels
    assert labels.get("amd.com/gpu.count") == "2" and labels.get("amd.com/gpu.arch") == "gfx950", labels
