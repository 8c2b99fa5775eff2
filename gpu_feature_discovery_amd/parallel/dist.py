"""Rank group for multi-process runs (one process per GPU).

``bench.py`` is launched by ``torch.distributed.run`` with one rank per GPU
(RANK / WORLD_SIZE / MASTER_ADDR from the environment).  The labeler itself
never communicates - feature discovery is a per-node job - so the ranks only
need to agree on the backend, bracket the timed region with barriers and
take the MAX of their wall times.  That is control-plane traffic of a few
bytes, so it rides on ``gloo`` over 127.0.0.1; RCCL would need a HIP context
in every rank, and a process that holds ``/dev/kfd`` makes ``amdsmi_init``
~100x cheaper than the real daemon ever sees (measured 26 ms -> 0.2 ms),
which would falsify the measurement.
"""

from __future__ import annotations

import os

__all__ = ["RankGroup", "env_int"]


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


class RankGroup:
    """Barrier / max-reduce across ranks (gloo), or no-ops for one process."""

    def __init__(self):
        self.world = env_int("WORLD_SIZE", 1)
        self.rank = env_int("RANK", 0)
        self.torch = None
        self.dist = None
        # One process: nothing to rendezvous with, so PyTorch is not loaded at
        # all - the production daemon never has it in its address space, and
        # its mere presence (threads, a second libdrm) slows amd-smi queries
        # by ~6 us per cycle (profiles/inproc_trace.txt).
        if self.world > 1:
            import torch
            import torch.distributed as dist

            self.torch = torch

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def sync(self):
        if self.dist is not None:
            self.dist.barrier()
        # The labeler issues no GPU work, so there is nothing to wait for; and
        # creating a HIP context here would change what is measured: a process
        # that already holds /dev/kfd makes amdsmi_init ~100x cheaper
        # (measured: 26 ms -> 0.2 ms), which the real daemon never sees.
        # Synchronize only if something else initialised the device.
        if self.torch is not None and self.torch.cuda.is_initialized():
            self.torch.cuda.synchronize()

    def max(self, v: float) -> float:
        if self.dist is None:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def broadcast_obj(self, obj):
        if self.dist is None:
            return obj
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=0)
        return lst[0]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
