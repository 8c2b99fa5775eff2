"""Packaging checks (reference analogue: tests/check-yamls.sh and the
static/Helm manifests under deployments/).  Every manifest is parsed with the
daemon's own YAML reader; image tags and version labels must match
versions.mk, env var names must be flags the daemon understands, and the
Helm templates may only reference values that exist."""

from __future__ import annotations

import os
import re
from pathlib import Path

import pytest

from conftest import REPO

DEPLOY = REPO / "deployments"
STATIC = DEPLOY / "static"
CHART = DEPLOY / "helm" / "gpu-feature-discovery-amd"


def _version() -> str:
    m = re.search(r"^VERSION \?= (v[0-9.]+)", (REPO / "versions.mk").read_text(), re.M)
    assert m
    return m.group(1)


def _docs(native, path: Path) -> list:
    text = path.read_text()
    return [native.parse_yaml(d) for d in re.split(r"^---\s*$", text, flags=re.M) if d.strip()]


def _env_vars(native) -> set[str]:
    help_text = __import__("subprocess").run([str(REPO / "build" / "gpu-feature-discovery"), "--help"],
                                             capture_output=True, text=True).stdout
    return set(re.findall(r"\$([A-Z_]+)", help_text))


@pytest.mark.parametrize("name,strategy", [
    ("gpu-feature-discovery-daemonset.yaml", "none"),
    ("gpu-feature-discovery-daemonset-with-partition-single.yaml", "single"),
    ("gpu-feature-discovery-daemonset-with-partition-mixed.yaml", "mixed"),
])
def test_static_daemonsets(native, name, strategy):
    (ds,) = _docs(native, STATIC / name)
    assert ds["kind"] == "DaemonSet"
    v = _version()
    assert ds["metadata"]["labels"]["app.kubernetes.io/version"] == v.lstrip("v")
    spec = ds["spec"]["template"]["spec"]
    (c,) = spec["containers"]
    assert c["image"].endswith(":" + v)
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["GFD_MIG_STRATEGY"] == strategy
    assert set(env) <= _env_vars(native)
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert {"/etc/kubernetes/node-feature-discovery/features.d", "/sys", "/host/opt"} <= mounts
    _check_host_opt(spec, c)
    assert env["GFD_HOST_ROOT"] == "/host"
    terms = spec["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"]["nodeSelectorTerms"]
    keys = {e["key"] for t in terms for e in t["matchExpressions"]}
    assert "feature.node.kubernetes.io/pci-1002.present" in keys


def _check_host_opt(spec, container):
    """The node's ROCm release comes from the host's /opt (read-only), which
    --host-root=/host points the daemon at - never from the image."""
    vols = {v["name"]: v for v in spec["volumes"]}
    assert vols["host-opt"]["hostPath"]["path"] == "/opt"
    # Directory, not DirectoryOrCreate: the labeler never writes to the host
    # (a node without /opt fails to mount, visibly).
    assert vols["host-opt"]["hostPath"]["type"] == "Directory"
    (m,) = [m for m in container["volumeMounts"] if m["name"] == "host-opt"]
    assert m["mountPath"] == "/host/opt" and m["readOnly"] is True


def test_job_template(native):
    (job,) = _docs(native, STATIC / "gpu-feature-discovery-job.yaml.template")
    spec = job["spec"]["template"]["spec"]
    assert spec["nodeName"] == "NODE_NAME"
    assert spec["restartPolicy"] == "Never"
    args = spec["containers"][0]["args"]
    assert "--oneshot" in args and "--backend=auto" in args and "--host-root=/host" in args
    assert spec["containers"][0]["image"].endswith(":" + _version())
    _check_host_opt(spec, spec["containers"][0])


def test_nfd_manifest(native):
    docs = _docs(native, STATIC / "nfd.yaml")
    kinds = [d["kind"] for d in docs]
    assert {"Namespace", "Deployment", "DaemonSet", "ConfigMap"} <= set(kinds)
    master = next(d for d in docs if d["kind"] == "Deployment")
    assert "-extra-label-ns=amd.com" in master["spec"]["template"]["spec"]["containers"][0]["args"]
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    conf = native.parse_yaml(cm["data"]["nfd-worker.conf"])
    assert "12" in conf["sources"]["pci"]["deviceClassWhitelist"]


def test_helm_chart(native):
    chart = native.parse_yaml((CHART / "Chart.yaml").read_text())
    assert "v" + chart["appVersion"] == _version()
    values = native.parse_yaml((CHART / "values.yaml").read_text())
    assert values["migStrategy"] in ("none", "single", "mixed")
    assert values["nfd"]["master"]["extraLabelNs"] == ["amd.com"]
    referenced = set()
    for t in (CHART / "templates").iterdir():
        referenced |= set(re.findall(r"\.Values\.([A-Za-z]+)", t.read_text()))
    missing = referenced - set(values) - {"namespace"}  # validation.yml rejects `namespace`
    assert not missing, missing


def test_helm_env_names_are_daemon_flags(native):
    # The DaemonSet takes its env list from the gfd-amd.env helper.
    assert 'include "gfd-amd.env"' in (CHART / "templates" / "daemonset.yml").read_text()
    text = (CHART / "templates" / "_helpers.tpl").read_text()
    names = set(re.findall(r'"(GFD_[A-Z_]+)"', text)) | set(re.findall(r"name: (GFD_[A-Z_]+)", text))
    assert {"GFD_MIG_STRATEGY", "GFD_SLEEP_INTERVAL", "GFD_FAIL_ON_INIT_ERROR"} <= names
    assert names <= _env_vars(native)


def test_dockerfile(native):
    text = (DEPLOY / "container" / "Dockerfile").read_text()
    assert 'ENTRYPOINT ["/usr/bin/gpu-feature-discovery"]' in text
    assert "gfd_unit_tests" in text  # the build stage runs the unit tests
    # The image must not carry a ROCm version of its own (node-true labels).
    assert not re.search(r"^COPY .*\.info/version", text, re.M)


def test_devel_image_has_what_the_make_targets_run():
    """docker/Dockerfile.devel (the `make docker-<target>` / `make shell`
    image) starts from the image build stage's base and installs every tool
    a Makefile target calls."""
    import sys

    sys.path.insert(0, str(REPO / "tests" / "e2e" / "fakes"))
    import _image

    (devel,) = _image._stages((REPO / "docker" / "Dockerfile.devel").read_text())
    build_stage = _image._stages((DEPLOY / "container" / "Dockerfile").read_text())[0]
    assert devel["base"] == build_stage["base"]
    runs = " ".join(a for i, a in devel["steps"] if i == "RUN")
    for tool in ("cmake", "ninja-build", "g++", "clang", "clang-format", "python3-pybind11", "pytest",
                 "pytest-timeout", "pyyaml", "hypothesis", "pyflakes"):
        assert re.search(r"(^|\s)" + re.escape(tool) + r"(\s|$)", runs), tool
    make = (REPO / "Makefile").read_text()
    assert "docker-%: .build-image" in make and "shell: .build-image" in make


def test_docker_context_leaves_build_trees_out():
    """`make image` sends the repository root as the build context; a local
    build tree in it would reach the build stage's /src, where CMake refuses
    a cache made for another source path (`cmake -B build` fails)."""
    import sys

    sys.path.insert(0, str(REPO / "tests" / "e2e" / "fakes"))
    import _image

    files = _image.context_files()
    assert "CMakeLists.txt" in files and "deployments/container/Dockerfile" in files
    assert not [f for f in files if f.split("/")[0] in (".git", "gpurun_out") or f.startswith("build")]
    assert not [f for f in files if f.endswith((".so", ".o", ".a", ".pyc"))]


def test_image_holds_what_the_dockerfile_copies(image):
    """The runtime stage assembled from the Dockerfile (tests/e2e/fakes/_image.py):
    the daemon at its ENTRYPOINT, amd-smi under ROCM_PATH, libdrm_amdgpu and
    its marketing-name table, a base C/C++ runtime - and no ROCm version
    file, so rocm.runtime.* can only come from the host mount."""
    assert (image / "usr/bin/gpu-feature-discovery").is_file()
    assert list((image / "opt/rocm/lib").glob("libamd_smi.so.*"))
    assert (image / "usr/share/libdrm/amdgpu.ids").is_file()
    for lib in ("libdrm_amdgpu.so.1", "libdrm.so.2", "libc.so.6", "libstdc++.so.6", "libgcc_s.so.1"):
        assert (image / "usr/lib/x86_64-linux-gnu" / lib).exists(), lib
    assert not (image / "opt/rocm/.info/version").exists()
    assert (image / ".image.entrypoint").read_text().split() == ["/usr/bin/gpu-feature-discovery"]


def test_image_lacking_a_library_is_caught(image, tmp_path):
    """What the image check relies on: with libstdc++ removed from (a copy
    of) the image, loading amd-smi has to reach past the image - the loader's
    last resort is the host's system directories, there being no mount
    namespace - and the loader trace names that library as foreign."""
    import shutil
    import subprocess
    import sys

    sys.path.insert(0, str(REPO / "tests" / "e2e" / "fakes"))
    import _image

    broken = tmp_path / "image"
    shutil.copytree(image, broken, symlinks=True)
    for f in (broken / "usr/lib/x86_64-linux-gnu").glob("libstdc++.so.6*"):
        f.unlink()
    trace = tmp_path / "ld"
    argv, env = _image.command(broken, ["--oneshot", "--backend=amdsmi", f"--output-file={tmp_path / 'out'}"], {},
                               base={"PATH": "/usr/bin:/bin"}, trace=trace)
    subprocess.run(argv, env=env, capture_output=True, text=True, timeout=60)
    assert [os.path.basename(o) for o in _image.foreign_libraries(broken, trace)] == ["libstdc++.so.6"]
    assert not _image.foreign_libraries(image, _trace_of_intact_run(image, tmp_path))


def _trace_of_intact_run(image, tmp_path):
    import subprocess
    import sys

    sys.path.insert(0, str(REPO / "tests" / "e2e" / "fakes"))
    import _image

    trace = tmp_path / "ld-intact"
    argv, env = _image.command(image, ["--oneshot", "--backend=amdsmi", f"--output-file={tmp_path / 'out-intact'}"], {},
                               base={"PATH": "/usr/bin:/bin"}, trace=trace)
    subprocess.run(argv, env=env, capture_output=True, text=True, timeout=60)
    assert _image.matches(_image.loaded_objects(trace), "libamd_smi.so*")
    return trace


def test_helm_mounts_host_opt(native):
    text = (CHART / "templates" / "daemonset.yml").read_text()
    assert "mountPath: /host/opt, readOnly: true" in text
    values = native.parse_yaml((CHART / "values.yaml").read_text())
    assert values["hostOpt"] == {"enabled": True, "path": "/opt"}
    assert "GFD_HOST_ROOT" in (CHART / "templates" / "_helpers.tpl").read_text()


def test_ci_workflow_runs_what_the_readme_claims(native):
    """The oracle suite must run (not skip) in CI, and the image job must run
    the image it built (round-1 review: neither happened)."""
    (wf,) = _docs(native, REPO / ".github" / "workflows" / "ci.yml")
    steps = [s.get("run", "") for s in wf["jobs"]["build-test"]["steps"]]
    assert any("hypothesis" in s and "pyyaml" in s for s in steps)
    assert any(s.startswith("CI=1 make test") for s in steps)
    image = " ".join(s.get("run", "") for s in wf["jobs"]["image"]["steps"])
    assert "docker run" in image and "--oneshot --backend=null" in image
    assert "test -e /opt/rocm/.info/version" in image


def test_chart_dependencies_are_in_the_repository(native):
    """An offline `helm install` of the default values needs every
    dependency in charts/ (the reference vendors NFD's chart as a .tgz;
    Chart.yaml:10-15): no remote repository, and name/version match."""
    chart = native.parse_yaml((CHART / "Chart.yaml").read_text())
    for dep in chart["dependencies"]:
        assert dep["repository"].startswith("file://"), dep
        sub = CHART / dep["repository"][len("file://"):]
        meta = native.parse_yaml((sub / "Chart.yaml").read_text())
        assert (meta["name"], meta["version"]) == (dep["name"], dep["version"])
    values = native.parse_yaml((CHART / "values.yaml").read_text())
    assert values["nfd"]["deploy"] is True  # deployable by default: it is in the repository


def _render(values=None, namespace="gpu-feature-discovery"):
    import helm_lite

    return helm_lite.documents(helm_lite.render_chart(CHART, values, namespace=namespace))


def test_chart_renders_offline_from_the_default_values(native):
    """`helm template` of the chart's defaults, done by tests/helm_lite.py:
    the labeler DaemonSet plus the in-repo NFD subchart, and what labeling
    depends on - the labeler's env are daemon flags, it mounts features.d,
    /sys and the host's /opt; NFD publishes amd.com, reads the same
    features.d and whitelists the accelerator PCI class, on the gRPC path."""
    docs = _render()
    kinds = sorted(d["kind"] for d in docs)
    assert kinds == ["ClusterRole", "ClusterRoleBinding", "ConfigMap", "DaemonSet", "DaemonSet", "Deployment",
                     "Service", "ServiceAccount"]
    (gfd,) = [d for d in docs if d["kind"] == "DaemonSet" and d["metadata"]["name"] == "gfd-gpu-feature-discovery-amd"]
    spec = gfd["spec"]["template"]["spec"]
    (c,) = spec["containers"]
    env = {e["name"]: e["value"] for e in c["env"]}
    assert set(env) <= _env_vars(native), set(env) - _env_vars(native)
    assert env["GFD_MIG_STRATEGY"] == "none" and env["GFD_HOST_ROOT"] == "/host"
    assert c["image"].endswith(":" + _version())
    vols = {v["name"]: v["hostPath"] for v in spec["volumes"]}
    assert vols["host-opt"] == {"path": "/opt", "type": "Directory"}
    assert spec["priorityClassName"] == "system-node-critical"
    master = next(d for d in docs if d["kind"] == "Deployment")
    args = master["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "-extra-label-ns=amd.com" in args and "-enable-nodefeature-api=false" in args
    (worker,) = [d for d in docs if d["kind"] == "DaemonSet" and d["metadata"]["name"] == "gfd-nfd-worker"]
    wspec = worker["spec"]["template"]["spec"]
    assert "-server=gfd-nfd-master:8080" in wspec["containers"][0]["args"]
    assert {"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"} in wspec["tolerations"]
    wvols = {v["name"]: v for v in wspec["volumes"]}
    assert wvols["features-d"]["hostPath"]["path"] == vols["features-d"]["path"]
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    conf = native.parse_yaml(cm["data"]["nfd-worker.conf"])
    assert "12" in conf["sources"]["pci"]["deviceClassWhitelist"]


def test_chart_takes_the_references_nfd_values(native):
    """A values file written for the reference's chart names its bundled NFD
    objects with nfd.nameOverride and nfd.master.serviceAccount.name
    (deployments/helm/gpu-feature-discovery/values.yaml:68-74); the in-repo
    NFD subchart takes both."""
    docs = _render({"nfd": {"nameOverride": "node-feature-discovery",
                            "master": {"serviceAccount": {"name": "node-feature-discovery"}}}})
    names = {(d["kind"], d["metadata"]["name"]) for d in docs}
    assert ("Deployment", "gfd-node-feature-discovery-master") in names
    assert ("DaemonSet", "gfd-node-feature-discovery-worker") in names
    assert ("ServiceAccount", "node-feature-discovery") in names
    master = next(d for d in docs if d["kind"] == "Deployment")
    assert master["spec"]["template"]["spec"]["serviceAccountName"] == "node-feature-discovery"
    binding = next(d for d in docs if d["kind"] == "ClusterRoleBinding")
    assert binding["subjects"][0]["name"] == "node-feature-discovery"
    (worker,) = [d for d in docs if d["kind"] == "DaemonSet" and "worker" in d["metadata"]["name"]]
    assert "-server=gfd-node-feature-discovery-master:8080" in worker["spec"]["template"]["spec"]["containers"][0]["args"]
    # The reference's extraLabelNs (nvidia.com) still lets amd.com through.
    docs = _render({"nfd": {"master": {"extraLabelNs": ["nvidia.com"]}}})
    args = next(d for d in docs if d["kind"] == "Deployment")["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "-extra-label-ns=nvidia.com" in args and "-extra-label-ns=amd.com" in args


def test_chart_options_render(native):
    """nfd.deploy=false drops the subchart; a config file becomes a ConfigMap,
    a mount, GFD_CONFIG_FILE and a checksum annotation (pods restart when it
    changes); an unprivileged pod (securityContext: null - an empty map would
    be merged with the default) drops every capability."""
    docs = _render({"nfd": {"deploy": False}, "config": {"version": "v1", "flags": {"migStrategy": "mixed"}},
                    "securityContext": None})
    assert sorted(d["kind"] for d in docs) == ["ConfigMap", "DaemonSet"]
    (ds,) = [d for d in docs if d["kind"] == "DaemonSet"]
    pod = ds["spec"]["template"]
    assert "checksum/config" in pod["metadata"]["annotations"]
    (c,) = pod["spec"]["containers"]
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["GFD_CONFIG_FILE"] == "/etc/gfd/config.yaml"
    assert {"name": "gfd-config", "mountPath": "/etc/gfd", "readOnly": True} in c["volumeMounts"]
    assert c["securityContext"] == {"allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}}
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    assert native.parse_yaml(cm["data"]["config.yaml"])["flags"]["migStrategy"] == "mixed"


@pytest.mark.parametrize("values,namespace,message", [
    ({"namespace": "x"}, "gpu-feature-discovery", "'namespace' value is not supported"),
    ({}, "default", "'default' namespace is not allowed"),
    ({"migStrategy": "bogus"}, "gpu-feature-discovery", "migStrategy must be one of"),
])
def test_chart_validation_fails_like_the_reference(values, namespace, message):
    """templates/validation.yml (reference: templates/validation.yml:1-16)."""
    import helm_lite

    with pytest.raises(helm_lite.HelmFail, match=message):
        _render(values, namespace=namespace)
    if namespace == "default":
        _render({"allowDefaultNamespace": True}, namespace="default")


def test_helm_lite_refuses_what_it_does_not_implement():
    import helm_lite

    with pytest.raises(helm_lite.HelmFail, match="unsupported function"):
        helm_lite.render("{{ lower .Values.x }}", {"x": "A"})
    with pytest.raises(helm_lite.HelmFail, match="no template"):
        helm_lite.render('{{ include "x" . }}', {})
    assert helm_lite.render("{{ .Values.missing }}", {}) == ""  # Helm renders a missing key empty
    assert helm_lite.render("a:{{- range .Values.l }} {{ . }}{{- end }}", {"l": [1, 2]}) == "a: 1 2"
    assert helm_lite.render('{{ if and .Values.a (not .Values.b) }}y{{ else }}n{{ end }}', {"a": 1, "b": 0}) == "y"


# ---- The manifests' own argv / env / mounts, run (tests/manifest_pods.py) --

MANIFEST_PODS = [
    ("static-daemonset", "gpu-feature-discovery-daemonset.yaml", "none"),
    ("static-daemonset-single", "gpu-feature-discovery-daemonset-with-partition-single.yaml", "single"),
    ("static-daemonset-mixed", "gpu-feature-discovery-daemonset-with-partition-mixed.yaml", "mixed"),
    ("static-job", "gpu-feature-discovery-job.yaml.template", "none"),
    ("helm", None, "none"),
]


def manifest_pod(native, source):
    import manifest_pods

    return manifest_pods.from_helm(CHART) if source is None else manifest_pods.from_static(native, STATIC / source)


def check_manifest_run(r, pod, strategy, rocm: str):
    """What every manifest run must show: exit 0, the full-GPU label set
    (regex golden, both directions), the node's ROCm release, and the
    DaemonSet removing its file at exit (main.go:149-156) / the Job not."""
    from gpu_feature_discovery_amd.utils import golden

    assert r["rc"] == 0, r["stderr"][-3000:]
    assert r["text"], r["stderr"][-3000:]
    labels = golden.parse_labels(r["text"])
    assert labels.get("amd.com/partition.strategy", "none") == strategy
    golden.check_regex_golden(r["text"], REPO / "tests" / "expected-output.txt",
                              select=lambda ln: not ln.startswith("amd.com/partition.strategy="))
    major, minor = rocm.split(".")[:2]
    assert (labels["amd.com/rocm.runtime.major"], labels["amd.com/rocm.runtime.minor"]) == (major, minor)
    assert r["removed_at_exit"] == (pod.kind == "DaemonSet")
    # Started from the image's own files: every library it loaded is the
    # image's (none came from the host's library directories).
    assert r["loaded"] and not r["foreign"], r["foreign"]


@pytest.mark.parametrize("name,source,strategy", MANIFEST_PODS, ids=[m[0] for m in MANIFEST_PODS])
def test_manifest_pod_runs_on_a_synthetic_node(native, image, tmp_path, name, source, strategy):
    """CPU rehearsal of tests/test_gpu.py::test_manifest_pod_labels_the_real_node:
    the same argv/env/mounts over a synthetic MI355X tree (the only added
    setting is --sysfs-root, since this container's /sys has no GPU)."""
    import manifest_pods
    from gpu_feature_discovery_amd.utils import synth

    pod = manifest_pod(native, source)
    root = synth.make_mi355x_node(tmp_path / "node", n_gpus=1, rocm_version="6.4.2", seed=40)
    croot = tmp_path / "container"
    manifest_pods.materialise(pod, croot, host_opt=root / "opt")
    r = manifest_pods.run(pod, image, croot, sysfs_root=str(root), timeout=60)
    check_manifest_run(r, pod, strategy, "6.4.2")


def test_manifest_pod_catches_a_broken_mount(native, image, tmp_path):
    """The point of running the manifests: the host /opt mounted somewhere
    --host-root does not look fails the run instead of dropping labels."""
    import manifest_pods
    from gpu_feature_discovery_amd.utils import synth

    pod = manifest_pod(native, "gpu-feature-discovery-daemonset.yaml")
    pod.mounts = {("/hostfs/opt" if m == "/host/opt" else m): h for m, h in pod.mounts.items()}
    root = synth.make_mi355x_node(tmp_path / "node", n_gpus=1, seed=41)
    croot = tmp_path / "container"
    manifest_pods.materialise(pod, croot, host_opt=root / "opt")
    r = manifest_pods.run(pod, image, croot, sysfs_root=str(root), timeout=30)
    assert r["rc"] == 1 and "has no opt/ directory" in r["stderr"]
