"""Replays the fuzz corpus (tests/fuzz/corpus: seeds and every input that
once crashed a target) through the fuzz targets linked with a plain driver,
so a regression of a fuzzer-found bug fails the CPU suite without libFuzzer.
Under `make asan` the same targets run with ASan/UBSan (build-asan)."""

from __future__ import annotations

import os
import subprocess

import pytest

from conftest import REPO

CORPUS = REPO / "tests" / "fuzz" / "corpus"


@pytest.mark.parametrize("target", ["config", "pci", "values", "flags", "sysfs", "amdsmi"])
def test_fuzz_corpus_replays_cleanly(target):
    build = os.environ.get("GFD_BUILD_DIR", str(REPO / "build"))
    exe = os.path.join(build, f"fuzz_replay_{target}")
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built")
    cp = subprocess.run([exe, str(CORPUS / target)], capture_output=True, text=True, timeout=120,
                        env={**os.environ, "UBSAN_OPTIONS": "halt_on_error=1"})
    assert cp.returncode == 0, cp.stdout[-2000:] + cp.stderr[-3000:]
    assert "replayed" in cp.stdout
