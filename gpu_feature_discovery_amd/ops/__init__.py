"""Operations of the daemon, callable in-process: :class:`Labeler` (a
configured instance running labeling cycles), :func:`label_once`,
:func:`devices`."""

from .labeling import CycleResult, Labeler, devices, label_once

__all__ = ["CycleResult", "Labeler", "devices", "label_once"]
