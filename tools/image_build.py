#!/usr/bin/env python3
"""`docker build` of deployments/container/Dockerfile without docker: the
build stage run for real (the .dockerignore'd context copied to its WORKDIR,
its RUN steps - CMake build, C++ unit tests, CPU pytest suite - executed,
package installs skipped), then the runtime stage assembled from that
stage's output (tests/e2e/fakes/_image.py), then the image's ENTRYPOINT run
with `--version` and a oneshot over a synthetic MI355X node, through the
image's own loader, and its loaded libraries checked.

    python tools/image_build.py [--work DIR]
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests" / "e2e" / "fakes"))

import _image  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--work", default=None, help="scratch directory (default: a new temporary one)")
    a = ap.parse_args()
    work = Path(a.work or tempfile.mkdtemp(prefix="gfd-docker-build-"))
    print(f"# build context: {len(_image.context_files())} files after .dockerignore", flush=True)
    t0 = time.monotonic()
    # As the container Makefile passes it (versions.mk's GIT_COMMIT).
    commit = subprocess.run(["git", "-C", str(REPO), "describe", "--match=", "--dirty", "--long", "--always"],
                            capture_output=True, text=True).stdout.strip() or "unknown"
    src = _image.run_build_stage(work / "build-stage", log=lambda m: print(f"# {m}", flush=True),
                                 build_args={"GIT_COMMIT": commit})
    print(f"# build stage: ok in {time.monotonic() - t0:.0f} s", flush=True)
    root = _image.build(work / "image", build_src=src)
    size = subprocess.run(["du", "-sh", str(root)], capture_output=True, text=True).stdout.split()[0]
    print(f"# runtime stage: {root} ({size})", flush=True)

    from gpu_feature_discovery_amd.utils import synth

    node = synth.make_mi355x_node(work / "node", n_gpus=8, seed=7)
    ok = True
    for name, args in (("--version", ["--version"]),
                       ("oneshot", ["--oneshot", "--no-timestamp", f"--sysfs-root={node}", "--host-root=" + str(node),
                                    f"--machine-type-file={node}/sys/class/dmi/id/product_name",
                                    f"--output-file={work / 'labels'}"])):
        trace = work / f"ld-{name.strip('-')}"
        argv, env = _image.command(root, args, {}, base=dict(os.environ), trace=trace)
        cp = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=60)
        foreign = _image.foreign_libraries(root, trace)
        loaded = [os.path.relpath(o, root) for o in _image.loaded_objects(trace)]
        print(f"{name}: exit {cp.returncode}; loaded from the image: {loaded}; from the host: {foreign}")
        ok &= cp.returncode == 0 and not foreign
        if name == "--version":
            print("   " + cp.stdout.strip().replace("\n", "\n   "))
            ok &= f"commit: {commit}" in cp.stdout
    labels = (work / "labels").read_text().splitlines()
    print(f"oneshot labels ({len(labels)}): " + ", ".join(x for x in labels if "gpu.count" in x or "product" in x))
    if not a.work:
        shutil.rmtree(work, ignore_errors=True)
    print("IMAGE BUILD " + ("PASSED" if ok else "FAILED"))
    return 0 if ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
