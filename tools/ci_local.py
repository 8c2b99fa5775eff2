#!/usr/bin/env python3
"""Run the CI workflow's jobs locally, the way GitHub Actions would on a
fresh checkout: `.github/workflows/ci.yml` is parsed, the commit is checked
out into a clean worktree (actions/checkout), and each job's `run:` steps
execute in order with bash -e, stopping at the first failure.  Package
installs (`apt-get`, `pip3 install`) are skipped - there is no network, and
this image already has what they install; jobs that need docker or the GPU
runner are skipped too.  Prints one line per step and a verdict per job.

    python tools/ci_local.py [--rev HEAD] [--jobs build-test,sanitizers]
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import yaml

REPO = Path(__file__).resolve().parent.parent
SKIP_PREFIXES = ("apt-get", "pip3 install", "pip install")


def steps_of(job: dict, matrix: dict) -> list[str]:
    out = []
    for s in job.get("steps", []):
        if "run" not in s:
            continue
        cmd = s["run"]
        for k, v in matrix.items():
            cmd = cmd.replace("${{ matrix.%s }}" % k, str(v))
        out.append(cmd)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rev", default="HEAD")
    ap.add_argument("--jobs", default="build-test,sanitizers")
    a = ap.parse_args()
    wf = yaml.safe_load((REPO / ".github/workflows/ci.yml").read_text())
    rev = subprocess.run(["git", "-C", str(REPO), "rev-parse", "--short", a.rev], capture_output=True, text=True,
                         check=True).stdout.strip()
    print(f"# .github/workflows/ci.yml at {rev}, run locally by tools/ci_local.py (installs skipped: no network)")
    failed = False
    for name in a.jobs.split(","):
        job = wf["jobs"][name]
        runs = [dict(zip(job["strategy"]["matrix"], combo)) for combo in
                zip(*job["strategy"]["matrix"].values())] if "strategy" in job else [{}]
        for matrix in runs:
            label = name + (f" ({', '.join(f'{k}={v}' for k, v in matrix.items())})" if matrix else "")
            with tempfile.TemporaryDirectory(prefix="gfd-ci-") as d:
                work = Path(d) / "src"
                subprocess.run(["git", "-C", str(REPO), "worktree", "add", "--detach", "-q", str(work), rev], check=True)
                ok = True
                try:
                    for cmd in steps_of(job, matrix):
                        if cmd.strip().startswith(SKIP_PREFIXES):
                            print(f"{label}: skip  {cmd.strip()}")
                            continue
                        t0 = time.monotonic()
                        # errors="replace": a fuzzer's log holds raw input bytes.
                        cp = subprocess.run(["bash", "-e", "-c", cmd], cwd=work, capture_output=True, text=True,
                                            errors="replace", env={**os.environ, "CI": os.environ.get("CI", "")})
                        dt = time.monotonic() - t0
                        tail = (cp.stdout + cp.stderr).strip().splitlines()[-1:] or [""]
                        print(f"{label}: {'ok  ' if cp.returncode == 0 else 'FAIL'}  {cmd.strip()}  "
                              f"({dt:.0f} s) | {tail[0][:160]}", flush=True)
                        if cp.returncode != 0:
                            print(cp.stdout[-3000:] + cp.stderr[-3000:], file=sys.stderr)
                            ok = False
                            break
                finally:
                    subprocess.run(["git", "-C", str(REPO), "worktree", "remove", "--force", str(work)], check=False)
                print(f"{label}: {'PASSED' if ok else 'FAILED'}")
                failed |= not ok
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
