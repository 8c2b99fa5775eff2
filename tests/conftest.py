"""Shared pytest setup.

* registers the ``gpu`` marker (tests that need a real MI355X; the driver
  runs ``-m "not gpu"`` on CPU and ``-m gpu`` on the GPU box),
* builds the native targets once per session if they are missing,
* provides helpers to run the daemon binary and synthetic sysfs trees.
"""

from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import gpu_feature_discovery_amd as gfd  # noqa: E402
from gpu_feature_discovery_amd.utils import build as gbuild  # noqa: E402
from gpu_feature_discovery_amd.utils import synth  # noqa: E402

TESTS = Path(__file__).resolve().parent
GOLDEN = TESTS / "golden"
FIXTURES = TESTS / "fixtures"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real AMD Instinct GPU (MI355X) and its driver")
    if not gbuild.is_built():
        gbuild.build()


@pytest.fixture(scope="session")
def native():
    return gfd.native()


@pytest.fixture(scope="session")
def binary() -> str:
    return str(gfd.binary_path())


@pytest.fixture(scope="session")
def image():
    """The labeler image's root file system: deployments/container/Dockerfile's
    runtime stage assembled offline (tests/e2e/fakes/_image.py)."""
    sys.path.insert(0, str(TESTS / "e2e" / "fakes"))
    import _image

    return _image.build()


@pytest.fixture()
def machine_file(tmp_path) -> str:
    """Fake DMI product name (main_test.go setupMachineFile)."""
    p = tmp_path / "machine-type"
    p.write_text("product-name\n")
    return str(p)


def run_daemon(binary: str, *args: str, env: dict | None = None, timeout: float = 30, check: bool = False,
               input_env: bool = False) -> subprocess.CompletedProcess:
    e = {k: v for k, v in os.environ.items() if not k.startswith(("GFD_", "MIG_STRATEGY", "FAIL_ON_INIT", "CONFIG_FILE"))}
    if env:
        e.update(env)
    cp = subprocess.run([binary, *args], capture_output=True, text=True, timeout=timeout, env=e)
    if check and cp.returncode != 0:
        raise AssertionError(f"daemon failed rc={cp.returncode}\nstdout:\n{cp.stdout}\nstderr:\n{cp.stderr}")
    return cp


@pytest.fixture()
def mi355x_node(tmp_path):
    """Factory for synthetic MI355X sysfs trees."""

    def make(n_gpus: int = 1, **kw):
        root = tmp_path / f"root-{n_gpus}-{len(list(tmp_path.iterdir()))}"
        return str(synth.make_mi355x_node(root, n_gpus=n_gpus, **kw))

    return make


def has_amd_gpu() -> bool:
    return os.path.exists("/dev/kfd")
