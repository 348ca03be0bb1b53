"""Framework-internal helpers (not part of the reference API surface).

* :mod:`.validation`     -- device-side deferred input validation flags.
* :mod:`.profiling`      -- roctx ranges around update / forward / compute / sync buckets for ``rocprofv3 --marker-trace``
  (``TORCHMETRICS_AMD_ROCTX=1``).
* :mod:`.deferred`       -- device-side warnings / checks read together with the validation words.
* :mod:`.graphs`         -- HIP-graph capture of a metric's or collection's ``update`` / ``compute``.
* :mod:`.fused_compute`  -- eager one-launch ``MetricCollection.compute()`` (recorded task rows, no graph).
"""
from torchmetrics_amd.utils import validation  # noqa: F401
