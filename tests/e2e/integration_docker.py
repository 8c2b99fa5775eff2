#!/usr/bin/env python3
"""Container integration test on a real MI355X host.

Reference analogue: tests/integration-tests.py (runs the image privileged
with a temp dir bound to features.d, polls for the file, then checks the
labels bidirectionally against the regex goldens).  Needs docker and an AMD
GPU node; not part of the CPU test-suite.

    python3 tests/e2e/integration_docker.py IMAGE [--strategy none]
"""

from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))

from gpu_feature_discovery_amd.utils import golden  # noqa: E402


def check(text: str, strategy: str) -> None:
    """The labels against the regex golden of what the node is: an
    unpartitioned node gets the full-GPU set under every strategy (plus the
    strategy label under single/mixed); a partitioned one under `single`
    the node partition-single golden, under `mixed` per-profile resources."""
    labels = golden.parse_labels(text)
    assert labels.get("amd.com/partition.strategy", "none") == strategy, labels
    partitioned = labels.get("amd.com/gpu.compute-partition", "SPX") != "SPX"
    not_sriov = lambda ln: "sriov" not in ln  # noqa: E731
    if not partitioned or strategy == "none":
        golden.check_regex_golden(text, REPO / "tests" / "expected-output.txt",
                                  select=lambda ln: not_sriov(ln) and not ln.startswith("amd.com/partition.strategy="))
    elif strategy == "single":
        # The node golden: a real node keeps its ISA/topology labels (the
        # mock fixture's expected-output-partition-single.txt has none).
        golden.check_regex_golden(text, REPO / "tests" / "expected-output-partition-single-node.txt", select=not_sriov)
    else:
        per_profile = re.compile(r"amd\.com/partition-[a-z]+\.[0-9]+xcd\.[0-9]+gb\.(product|count|replicas|memory|"
                                 r"compute-units|xcds|compute-partition|memory-partition|engines\.[a-z]+)=[A-Za-z0-9_.-]+")
        keys = [k for k in labels if k.startswith("amd.com/partition-")]
        assert keys and all(per_profile.fullmatch(f"{k}={labels[k]}") for k in keys), keys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("image")
    ap.add_argument("--strategy", default="none")
    ap.add_argument("--timeout", type=float, default=60)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        name = f"gfd-amd-it-{int(time.time())}"
        subprocess.run(["docker", "run", "-d", "--rm", "--name", name, "--privileged",
                        "-v", f"{d}:/etc/kubernetes/node-feature-discovery/features.d",
                        "-v", "/sys:/sys:ro",
                        # The node's ROCm release, as the manifests provide it (the image has none).
                        "-v", "/opt:/host/opt:ro", "-e", "GFD_HOST_ROOT=/host",
                        "-e", f"GFD_MIG_STRATEGY={a.strategy}", "-e", "GFD_SLEEP_INTERVAL=5s",
                        a.image], check=True)
        try:
            out = Path(d) / "gfd"
            end = time.time() + a.timeout
            while not out.exists() and time.time() < end:
                time.sleep(1)
            if not out.exists():
                print("features.d/gfd never appeared", file=sys.stderr)
                return 1
            text = out.read_text()
            check(text, a.strategy)
            print(text, end="")
            print("integration test passed")
            return 0
        finally:
            subprocess.run(["docker", "stop", name], check=False, capture_output=True)


if __name__ == "__main__":
    sys.exit(main())
