"""Runs the C++ unit tests (tests/unit/*.cpp) and reports each one as its own
pytest case.  These are the ports of the reference's Go unit tests
(internal/lm/*_test.go, internal/vgpu/*_test.go, internal/resource/
fallback_test.go) plus the native parsers, backends and CLI."""

from __future__ import annotations

import subprocess

import pytest

import gpu_feature_discovery_amd as gfd


def _names() -> list[str]:
    out = subprocess.run([str(gfd.UNIT_TEST_BINARY), "--list"], capture_output=True, text=True, check=True).stdout
    return [n for n in out.splitlines() if n]


@pytest.fixture(scope="module")
def results() -> dict[str, str]:
    cp = subprocess.run([str(gfd.UNIT_TEST_BINARY)], capture_output=True, text=True, timeout=300)
    res: dict[str, str] = {}
    current = None
    for line in cp.stdout.splitlines():
        if line.startswith("[ OK ] "):
            res[line[7:]] = "ok"
            current = None
        elif line.startswith("[FAIL] "):
            current = line[7:]
            res[current] = ""
        elif current is not None:
            res[current] += line + "\n"
    return res


@pytest.mark.parametrize("name", _names())
def test_cpp(name, results):
    assert name in results, f"{name} did not run"
    assert results[name] == "ok", results[name]
