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
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))

from gpu_feature_discovery_amd.utils import golden  # noqa: E402


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
            goldens = {"none": "expected-output.txt", "single": "expected-output-partition-single.txt",
                       "mixed": "expected-output-partition-mixed.txt"}
            golden.check_regex_golden(text, REPO / "tests" / goldens[a.strategy], select=lambda ln: "sriov" not in ln)
            print(text, end="")
            print("integration test passed")
            return 0
        finally:
            subprocess.run(["docker", "stop", name], check=False, capture_output=True)


if __name__ == "__main__":
    sys.exit(main())
