"""MI355X-native GPU feature discovery.

The daemon is a native C++ binary (``build/gpu-feature-discovery``); this
package holds the Python side used by the test-suite and ``bench.py``:

* :mod:`._gfd` - pybind11 extension over the same native core (in-process
  labeling cycles, YAML/config parsing, device enumeration),
* :mod:`.ops` - typed in-process API over it (:class:`~.ops.Labeler`),
* :mod:`.models` - the MI355X device model (geometry, partition profiles),
* :mod:`.parallel` - rank group for one-process-per-GPU runs (bench.py),
* :mod:`.utils` - synthetic sysfs trees, golden-file helpers, in-tree build.

Reference: Telemaco019/gpu-feature-discovery (NVIDIA GFD v0.7.0 fork); see
SURVEY.md for the component mapping.
"""

from __future__ import annotations

import importlib
import os
from pathlib import Path

REPO_ROOT = Path(__file__).resolve().parent.parent
PACKAGE_DIR = Path(__file__).resolve().parent
BUILD_DIR = REPO_ROOT / "build"
BINARY = BUILD_DIR / "gpu-feature-discovery"
UNIT_TEST_BINARY = BUILD_DIR / "gfd_unit_tests"

__all__ = ["native", "binary_path", "REPO_ROOT", "BINARY", "UNIT_TEST_BINARY"]

_native = None


def native():
    """Return the native extension module, failing loudly if it is missing.

    There is deliberately no pure-Python fallback: every code path the tests
    and the benchmark exercise must run the C++ core.
    """
    global _native
    if _native is None:
        try:
            _native = importlib.import_module(".{}".format("_gfd"), __name__)
        except ImportError as e:  # pragma: no cover - exercised only when unbuilt
            raise ImportError(
                "gpu_feature_discovery_amd._gfd is not built; run "
                "`python -c 'import __graft_entry__ as g; g.build()'` or `make`"
            ) from e
    return _native


def binary_path() -> Path:
    """Path of the daemon binary (built in-tree)."""
    override = os.environ.get("GFD_BINARY")
    path = Path(override) if override else BINARY
    if not path.exists():
        raise FileNotFoundError(f"{path} not built; run `make` or __graft_entry__.build()")
    return path
