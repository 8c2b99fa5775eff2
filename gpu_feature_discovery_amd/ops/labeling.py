"""Typed Python API over the native labeling core.

Every function here runs the C++ daemon code in-process through the
``_gfd`` extension (no Python re-implementation, no fallback): a
:class:`Labeler` is one configured daemon instance - config, device backend
(amd-smi / KFD sysfs / mock / null) and SR-IOV scanner built once, exactly as
the daemon's ``start`` does (reference: ``cmd/gpu-feature-discovery/main.go``
``start``/``run``) - and each :meth:`Labeler.cycle` is one labeling cycle of
its ``run`` loop.  Arguments are the daemon's own command-line flags.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Sequence

from .. import native

__all__ = ["CycleResult", "Labeler", "label_once", "devices"]


@dataclass
class CycleResult:
    labels: dict[str, str]
    phases_ms: list[tuple[str, float]] = field(default_factory=list)
    total_ms: float = 0.0
    rendered: str = ""

    @classmethod
    def from_native(cls, r: dict) -> "CycleResult":
        return cls(labels=dict(r["labels"]), phases_ms=[(k, v / 1e6) for k, v in r["phases"]],
                   total_ms=r["total_ns"] / 1e6, rendered=r["rendered"])


class Labeler:
    """A configured daemon instance (flags as on the command line)."""

    def __init__(self, args: Sequence[str] = (), env: dict[str, str] | None = None,
                 amdsmi_library_only: bool = False):
        """``env``: a private environment for flag resolution (instead of the
        process's); ``amdsmi_library_only``: the amd-smi backend answers every
        query through library calls (a cross-check of its attribute reads)."""
        self._session = native().Session(list(args), env, amdsmi_library_only)

    @property
    def backend(self) -> str:
        return self._session.backend

    @property
    def config_json(self) -> str:
        """The effective configuration, as the daemon logs it at start."""
        return self._session.config_json

    def devices(self) -> list[dict]:
        """One enumeration through the configured backend."""
        return self._session.devices()

    def cycle(self, write: bool = False) -> CycleResult:
        """One labeling cycle; ``write`` atomically rewrites the output file."""
        return CycleResult.from_native(self._session.cycle(write))

    def bench(self, steps: int, warmup: int = 0, write: bool = True, traced: bool = True) -> list[float]:
        """``warmup`` untimed cycles then ``steps`` timed ones, in a native
        loop (no Python between cycles); returns per-cycle milliseconds.
        ``traced``: record each cycle's phases (``bench_phases``); untraced
        cycles read no clock for them, as the daemon's without
        ``--trace-timing``."""
        return [ns / 1e6 for ns in self._session.bench(steps, warmup, write, traced)]

    def bench_phases(self) -> dict[str, list[float]]:
        """Per-phase milliseconds of the last traced ``bench`` call's timed cycles."""
        return {name: [ns / 1e6 for ns in v] for name, v in self._session.bench_phases().items()}


def label_once(args: Sequence[str] = ()) -> CycleResult:
    """Labels of one cycle, without writing the output file."""
    return Labeler(args).cycle(write=False)


def devices(args: Sequence[str] = ()) -> list[dict]:
    """Devices as the configured backend enumerates them."""
    return Labeler(args).devices()
