"""Framework-internal helpers (not part of the reference API surface).

* :mod:`.validation` -- device-side deferred input validation flags.
* :mod:`.profiling` -- roctx-style ranges for ``rocprofv3 --marker-trace`` and a lightweight timer.
* :mod:`.graphs`    -- HIP-graph capture of a metric's ``update`` for launch-bound loops.
"""
from torchmetrics_amd.utils import validation  # noqa: F401
