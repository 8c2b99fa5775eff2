"""Multi-process helpers: :class:`RankGroup` (barrier / max-reduce /
broadcast over gloo for one-rank-per-GPU runs)."""

from .dist import RankGroup, env_int

__all__ = ["RankGroup", "env_int"]
