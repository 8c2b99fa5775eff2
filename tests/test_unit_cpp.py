"""Runs the C++ unit tests (tests/unit/*.cpp) and reports each one as its own
pytest case.  These are the ports of the reference's Go unit tests
(internal/lm/*_test.go, internal/vgpu/*_test.go, internal/resource/
fallback_test.go) plus the native parsers, backends and CLI."""

from __future__ import annotations

import os
import subprocess

import pytest

import gpu_feature_discovery_amd as gfd


def _names() -> list[str]:
    out = subprocess.run([str(gfd.UNIT_TEST_BINARY), "--list"], capture_output=True, text=True, check=True).stdout
    return [n for n in out.splitlines() if n]


@pytest.fixture(scope="module")
def results() -> dict[str, str]:
    env = {k: v for k, v in os.environ.items() if k != "GFD_AMDSMI_LIBRARY"}
    cp = subprocess.run([str(gfd.UNIT_TEST_BINARY)], capture_output=True, text=True, timeout=300, env=env)
    return _parse(cp.stdout)


def _parse(stdout: str) -> dict[str, str]:
    res: dict[str, str] = {}
    current = None
    for line in stdout.splitlines():
        if line.startswith("[ OK ] "):
            res[line[7:]] = "ok"
            current = None
        elif line.startswith("[FAIL] "):
            current = line[7:]
            res[current] = ""
        elif current is not None:
            res[current] += line + "\n"
    return res


FAKE_PREFIXES = ("AmdSmiFake_", "AmdSmiFault_")


@pytest.fixture(scope="module")
def fake_results() -> dict[str, str]:
    """The AmdSmiFake_* / AmdSmiFault_* tests, run against the scriptable
    libamd_smi (without it they return early)."""
    fake = gfd.BUILD_DIR / "libfake_amdsmi.so"
    names = [n for n in _names() if n.startswith(FAKE_PREFIXES)]
    env = {**os.environ, "GFD_AMDSMI_LIBRARY": str(fake)}
    cp = subprocess.run([str(gfd.UNIT_TEST_BINARY), *names], capture_output=True, text=True, timeout=300, env=env)
    return _parse(cp.stdout)


@pytest.mark.parametrize("name", _names())
def test_cpp(name, results, fake_results):
    if name.startswith(FAKE_PREFIXES):
        results = fake_results
    assert name in results, f"{name} did not run"
    assert results[name] == "ok", results[name]
