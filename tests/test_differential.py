"""A long-lived daemon labels like a fresh process, after any node change.

The reference has no state across cycles: it builds its labelers and
initialises NVML anew every cycle (cmd/gpu-feature-discovery/main.go:160,
internal/lm/nvml.go:30-33).  This daemon keeps facts between cycles (listed
in docs/ARCHITECTURE.md, "What is kept between cycles"), so random sequences
of node changes (tests/differential.py: partition and NPS switches, VFs,
GPUs added and removed, module reloads, driver binding, /opt/rocm
repointed, the version file rewritten or replaced, DMI, unrelated uevents)
are applied to synthetic nodes and, after every change, the feature file of
long-lived sessions - KFD-sysfs and amd-smi (the fake library, which like
the real one only sees a changed node when it is initialised again), each
under the three strategies, and the DaemonSet's default `auto` (KFD first,
amd-smi once ready) - must equal a fresh `--oneshot` process's byte for
byte.

GFD_DIFF_SEQUENCES / GFD_DIFF_STEPS / GFD_DIFF_SEED size a longer run.  A
few scripted sequences (differential.scripted_sequences) run first: changes
the random ones reach too rarely to guard.
"""

from __future__ import annotations

import concurrent.futures
import os
import random

import pytest

import differential as dd
from gpu_feature_discovery_amd import BUILD_DIR

FAKE = BUILD_DIR / "libfake_amdsmi.so"
STRATEGIES = ("none", "single", "mixed")
BACKENDS = ("sysfs", "amdsmi")


def _run(binary: str, tmp_path, sequences: int, steps: int, seed: int) -> dict:
    rng = random.Random(seed)
    server = dd.LongLived(str(FAKE))
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=7)
    counts: dict[str, int] = {}
    compared = 0
    scripted = dd.scripted_sequences()
    try:
        for s in range(len(scripted) + sequences):
            root = tmp_path / f"n{s}"
            script = scripted[s][1] if s < len(scripted) else None
            live = dd.LiveNode(root, scripted[s][0] if script else dd.random_node(rng))
            # The DaemonSet's default backend too: KFD first, amd-smi once it is
            # ready and agrees; a fresh Job labels it from KFD.
            ids = [(b, st) for b in BACKENDS for st in STRATEGIES] + [("auto", "single")]
            out = {k: str(tmp_path / f"out-{s}-{k[0]}-{k[1]}" / "gfd") for k in ids}
            server.call(op="stage", spec=live.fake_spec())
            for k in ids:
                assert server.call(op="open", id=f"{k[0]}/{k[1]}", args=dd.daemon_args(root, *k, out[k]))["ok"]
            history = ["initial"]
            for step in range(len(script) + 1 if script else steps):
                if step:
                    history.append(script[step - 1](live) if script else dd.mutate(live, rng))
                    counts[history[-1]] = counts.get(history[-1], 0) + 1
                    server.call(op="stage", spec=live.fake_spec())
                env = {**os.environ, "GFD_AMDSMI_LIBRARY": str(FAKE), "GFD_FAKE_AMDSMI_SPEC": live.fake_spec()}
                futs = {k: pool.submit(dd.fresh, binary, dd.daemon_args(root, *k, out[k] + ".fresh"), out[k] + ".fresh",
                                       env) for k in ids}
                for k in ids:
                    got = server.call(op="cycle", id=f"{k[0]}/{k[1]}", out=out[k])
                    want = futs[k].result()
                    assert got == want, (f"sequence {s} step {step} {k}: after {history}\n"
                                         f"long-lived: {got}\nfresh: {want}")
                    compared += 1
            for k in ids:
                server.call(op="close", id=f"{k[0]}/{k[1]}")
            live.close()
    finally:
        pool.shutdown()
        server.close()
    return {"compared": compared, "changes": counts}


@pytest.mark.skipif(not FAKE.exists(), reason="libfake_amdsmi.so not built")
@pytest.mark.timeout(300)
def test_long_lived_sessions_label_like_a_fresh_process(binary, tmp_path):
    sequences = int(os.environ.get("GFD_DIFF_SEQUENCES", "200"))
    steps = int(os.environ.get("GFD_DIFF_STEPS", "5"))
    seed = int(os.environ.get("GFD_DIFF_SEED", "20261018"))
    r = _run(binary, tmp_path, sequences, steps, seed)
    scripted_steps = sum(len(script) + 1 for _, script in dd.scripted_sequences())
    assert r["compared"] == (sequences * steps + scripted_steps) * (len(STRATEGIES) * len(BACKENDS) + 1)
    # Every kind of change was exercised.
    assert set(r["changes"]) == {"partition", "nps", "vfs", "gpu_add", "gpu_remove", "module_reload", "rocm_repoint",
                                 "rocm_rewrite", "rocm_replace", "dmi", "bind", "uevent"}, r["changes"]
