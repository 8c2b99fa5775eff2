"""Device models: the hardware facts labels are derived from.

* :mod:`.mi355x` - AMD Instinct MI355X (gfx950 / CDNA4): PCI identity, CU/XCD
  geometry, HBM3E size, xGMI hive, compute/memory partition modes and the
  partition-profile naming rule.
"""

from . import mi355x

__all__ = ["mi355x"]
