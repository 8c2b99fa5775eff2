"""Run the daemon exactly as a deployment manifest would.

The reference's container integration test runs its image privileged against
a real node and matches the labels (tests/integration-tests.py:36-78).  There
is no container runtime, helm or kubectl here or on the GPU box, so the
stand-in takes the labeler container of a manifest - the static DaemonSet or
Job template, or the Helm chart's DaemonSet rendered with its default values
(tests/helm_lite.py) - and
runs the labeler image (the Dockerfile's runtime stage assembled offline,
tests/e2e/fakes/_image.py: the daemon started from the image's own files and
libraries) with that container's argv and environment, its hostPath mounts
reproduced under a scratch "container root":

* features.d (hostPath /etc/kubernetes/node-feature-discovery/features.d):
  an empty directory at the same container path;
* the host's /opt (for --host-root): the node's /opt/rocm/.info/version
  copied to the same container path;
* /sys must be mounted at /sys (the daemon reads it there); the GPU run uses
  the real one, the CPU rehearsal a synthetic tree (--sysfs-root, the one
  setting that is added).

Every path-valued setting (env or argument) is a container path and is
re-rooted under the scratch root; nothing else is changed, so a manifest
whose env names, arguments or mounts do not fit the daemon fails the run.
"""

from __future__ import annotations

import os
import re
import shutil
import signal
import subprocess
import sys
import time
from dataclasses import dataclass, field
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent / "e2e" / "fakes"))
import _image  # noqa: E402

FEATURES_D = "/etc/kubernetes/node-feature-discovery/features.d"
DEFAULT_OUTPUT = FEATURES_D + "/gfd"
# Settings whose value is a path inside the container.
_PATH_ENV = ("GFD_OUTPUT_FILE", "GFD_HOST_ROOT", "GFD_CONFIG_FILE", "CONFIG_FILE", "GFD_ROCM_VERSION_FILE",
             "GFD_MACHINE_TYPE_FILE")
_PATH_ARGS = ("--output-file=", "--output=", "-o=", "--host-root=", "--config-file=", "--rocm-version-file=",
              "--machine-type-file=")


@dataclass
class Pod:
    kind: str                          # DaemonSet | Job
    args: list[str] = field(default_factory=list)
    env: dict[str, str] = field(default_factory=dict)
    mounts: dict[str, str] = field(default_factory=dict)  # container path -> hostPath


def from_static(native, path: Path) -> Pod:
    docs = [native.parse_yaml(d) for d in re.split(r"^---\s*$", path.read_text(), flags=re.M) if d.strip()]
    (obj,) = [d for d in docs if d.get("kind") in ("DaemonSet", "Job")]
    return from_pod_spec(obj["kind"], obj["spec"]["template"]["spec"])


def from_pod_spec(kind: str, spec: dict) -> Pod:
    (c,) = [c for c in spec["containers"] if c["name"] == "labeler"]
    vols = {v["name"]: v["hostPath"]["path"] for v in spec["volumes"] if "hostPath" in v}
    return Pod(kind=kind, args=[str(a) for a in c.get("args", [])],
               env={e["name"]: str(e["value"]) for e in c.get("env", []) or []},
               mounts={m["mountPath"]: vols[m["name"]] for m in c.get("volumeMounts", []) if m["name"] in vols})


def from_helm(chart: Path, values: dict | None = None) -> Pod:
    """The chart's DaemonSet container as `helm template` renders it with
    values.yaml's defaults (tests/helm_lite.py)."""
    import helm_lite

    docs = helm_lite.documents(helm_lite.render_chart(chart, values))
    (ds,) = [d for d in docs if d["kind"] == "DaemonSet" and d["metadata"]["name"].endswith("gpu-feature-discovery-amd")]
    return from_pod_spec("DaemonSet", ds["spec"]["template"]["spec"])


def materialise(pod: Pod, croot: Path, host_opt: Path = Path("/opt")) -> None:
    """Reproduce the pod's hostPath mounts under `croot`."""
    for mpath, hpath in pod.mounts.items():
        if mpath == "/sys":
            assert hpath == "/sys", f"/sys is mounted from {hpath}"
            continue
        local = croot / mpath.lstrip("/")
        local.mkdir(parents=True, exist_ok=True)
        if hpath == FEATURES_D:
            continue
        if hpath == "/opt":
            src = host_opt / "rocm" / ".info" / "version"
            if src.exists():
                dst = local / "rocm" / ".info" / "version"
                dst.parent.mkdir(parents=True, exist_ok=True)
                shutil.copyfile(os.path.realpath(src), dst)
            continue
        raise AssertionError(f"unknown hostPath {hpath} mounted at {mpath}")


def plan(pod: Pod, image: Path, croot: Path, sysfs_root: str | None = None,
         trace: Path | None = None) -> tuple[list[str], dict[str, str], Path]:
    """argv, environment and the output file (local path) of the pod's run
    from the image rooted at `image` (`_image.build()`)."""
    env = {k: v for k, v in os.environ.items()
           if not k.startswith(("GFD_", "MIG_STRATEGY", "FAIL_ON_INIT", "CONFIG_FILE"))}
    penv = dict(pod.env)
    args = list(pod.args)
    output = DEFAULT_OUTPUT
    for k in _PATH_ENV:
        if k in penv:
            if k == "GFD_OUTPUT_FILE":
                output = penv[k]
            penv[k] = str(croot) + penv[k]
    for i, a in enumerate(args):
        for flag in _PATH_ARGS:
            if a.startswith(flag):
                if flag in ("--output-file=", "--output=", "-o="):
                    output = a[len(flag):]
                args[i] = flag + str(croot) + a[len(flag):]
    if not any(a.startswith(("--output-file=", "--output=", "-o=")) for a in args) and "GFD_OUTPUT_FILE" not in pod.env:
        penv["GFD_OUTPUT_FILE"] = str(croot) + output  # the default, re-rooted
    assert any(output.startswith(m + "/") and h == FEATURES_D for m, h in pod.mounts.items()), \
        f"the feature file {output} is not in the mounted features.d"
    if sysfs_root:
        penv["GFD_SYSFS_ROOT"] = sysfs_root
        penv.setdefault("GFD_MACHINE_TYPE_FILE", sysfs_root + "/sys/class/dmi/id/product_name")
    argv, env = _image.command(image, args, penv, base=env, trace=trace)
    return argv, env, croot / output.lstrip("/")


def run(pod: Pod, image: Path, croot: Path, sysfs_root: str | None = None, timeout: float = 120) -> dict:
    """Run the pod's labeler: a Job to completion; a DaemonSet until its first
    feature file, then SIGTERM (as a pod deletion does).  Returns the feature
    file, stderr, exit code, whether the file was removed at exit, and the
    shared objects the process loaded: all of them, and those that came from
    the host's library directories instead of the image."""
    trace = croot.parent / (croot.name + ".ld")
    argv, env, out = plan(pod, image, croot, sysfs_root, trace)

    def libraries() -> dict:
        return {"loaded": _image.loaded_objects(trace), "foreign": _image.foreign_libraries(image, trace)}

    if pod.kind == "Job":
        cp = subprocess.run(argv, capture_output=True, text=True, timeout=timeout, env=env)
        return {"text": out.read_text() if out.exists() else "", "stderr": cp.stderr, "rc": cp.returncode,
                "removed_at_exit": not out.exists(), **libraries()}
    p = subprocess.Popen(argv, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=env)
    text = ""
    try:
        end = time.monotonic() + timeout
        while time.monotonic() < end and p.poll() is None:
            if out.exists():
                text = out.read_text()
                break
            time.sleep(0.01)
    finally:
        p.send_signal(signal.SIGTERM)
        _, err = p.communicate(timeout=30)
    return {"text": text, "stderr": err, "rc": p.returncode, "removed_at_exit": not out.exists(), **libraries()}
