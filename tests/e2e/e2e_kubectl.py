#!/usr/bin/env python3
"""End-to-end test on a Kubernetes cluster with MI355X nodes.

Reference analogue: tests/e2e-tests.py (deploys NFD + the GFD DaemonSet and
waits up to 180 s for the timestamp label).  Unlike the reference, every
node carrying `feature.node.kubernetes.io/pci-1002.present=true` is checked,
not only nodes[0].  Needs kubectl with cluster-admin.

    python3 tests/e2e/e2e_kubectl.py [--image IMAGE] [--timeout 180] [--strategy none|single|mixed]

With --strategy the DaemonSet of that partition strategy is deployed
(deployments/static/gpu-feature-discovery-daemonset[-with-partition-*].yaml)
and each node's published amd.com labels are checked against the regex
goldens of what the node is, as the container integration test does.
"""

from __future__ import annotations

import argparse
import json
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
STATIC = REPO / "deployments" / "static"
sys.path.insert(0, str(Path(__file__).resolve().parent))

from integration_docker import check  # noqa: E402


def kubectl(*args: str, input_text: str | None = None) -> str:
    return subprocess.run(["kubectl", *args], check=True, capture_output=True, text=True, input=input_text).stdout


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", default=None)
    ap.add_argument("--timeout", type=float, default=180)
    ap.add_argument("--strategy", default=None, choices=["none", "single", "mixed"])
    a = ap.parse_args()
    kubectl("apply", "-f", str(STATIC / "nfd.yaml"))
    manifest = "gpu-feature-discovery-daemonset.yaml"
    if a.strategy in ("single", "mixed"):
        manifest = f"gpu-feature-discovery-daemonset-with-partition-{a.strategy}.yaml"
    ds = (STATIC / manifest).read_text()
    if a.image:
        ds = "\n".join(ln if "image:" not in ln else ln.split("image:")[0] + f"image: {a.image}" for ln in ds.splitlines())
    with tempfile.NamedTemporaryFile("w", suffix=".yaml") as f:
        f.write(ds)
        f.flush()
        kubectl("apply", "-f", f.name)
    end = time.time() + a.timeout
    pending = None
    while time.time() < end:
        nodes = json.loads(kubectl("get", "nodes", "-l", "feature.node.kubernetes.io/pci-1002.present=true", "-o",
                                   "json"))["items"]
        pending = [n["metadata"]["name"] for n in nodes if "amd.com/gfd.timestamp" not in n["metadata"]["labels"]]
        if nodes and not pending:
            for n in nodes:
                labels = {k: v for k, v in n["metadata"]["labels"].items() if k.startswith("amd.com/")}
                assert labels.get("amd.com/gpu.arch", "").startswith("gfx"), labels
                if a.strategy:
                    check("".join(f"{k}={v}\n" for k, v in sorted(labels.items())), a.strategy)
                print(n["metadata"]["name"], json.dumps(labels, indent=1, sort_keys=True))
            print("e2e test passed")
            return 0
        time.sleep(5)
    print(f"timed out; nodes without labels: {pending}", file=sys.stderr)
    return 1


if __name__ == "__main__":
    sys.exit(main())
