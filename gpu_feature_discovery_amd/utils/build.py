"""Build the native targets in-tree (CMake + Ninja).

Produces ``build/gpu-feature-discovery``, ``build/gfd_unit_tests`` and
``gpu_feature_discovery_amd/_gfd*.so``.  The daemon has no HIP kernels (the
reference launches no device code either), so no gfx950 code
object is built; amd-smi is dlopen'ed at runtime.
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

from .. import BUILD_DIR, REPO_ROOT


def _jobs() -> str:
    n = os.environ.get("MAX_JOBS") or os.environ.get("CMAKE_BUILD_PARALLEL_LEVEL")
    if not n:
        n = str(min(16, os.cpu_count() or 4))
    return n


def build(build_type: str = "Release", extra_cmake_args: list[str] | None = None, quiet: bool = True,
          build_dir: Path | None = None) -> None:
    bdir = Path(build_dir) if build_dir else BUILD_DIR
    generator = ["-G", "Ninja"] if shutil.which("ninja") else []
    cache = bdir / "CMakeCache.txt"
    if cache.exists() and generator and "Ninja" not in cache.read_text(errors="ignore"):
        shutil.rmtree(bdir)  # generator changed
    cmd = ["cmake", "-S", str(REPO_ROOT), "-B", str(bdir), f"-DCMAKE_BUILD_TYPE={build_type}",
           f"-DPython3_EXECUTABLE={sys.executable}", *generator, *(extra_cmake_args or [])]
    out = subprocess.DEVNULL if quiet else None
    subprocess.run(cmd, check=True, stdout=out)
    subprocess.run(["cmake", "--build", str(bdir), "-j", _jobs()], check=True, stdout=out)


def is_built() -> bool:
    from .. import BINARY, PACKAGE_DIR, UNIT_TEST_BINARY
    return (BINARY.exists() and UNIT_TEST_BINARY.exists() and (BUILD_DIR / "libfake_amdsmi.so").exists()
            and any(PACKAGE_DIR.glob("_gfd*.so")))


if __name__ == "__main__":
    build(quiet=False)
