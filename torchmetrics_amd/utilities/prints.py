"""Rank-zero gated logging (parity: reference ``S/utilities/prints.py:22-73``)."""
import logging
import os
import warnings
from functools import partial, wraps
from typing import Any, Callable, Optional

log = logging.getLogger("torchmetrics_amd")


def _local_rank() -> int:
    for key in ("LOCAL_RANK", "SLURM_LOCALID", "JSM_NAMESPACE_LOCAL_RANK"):
        if key in os.environ:
            try:
                return int(os.environ[key])
            except ValueError:
                pass
    return 0


def rank_zero_only(fn: Callable) -> Callable:
    """Run ``fn`` only on local rank 0; other ranks return ``None``."""

    @wraps(fn)
    def wrapped(*args: Any, **kwargs: Any) -> Optional[Any]:
        if rank_zero_only.rank == 0:
            return fn(*args, **kwargs)
        return None

    return wrapped


rank_zero_only.rank = _local_rank()  # type: ignore[attr-defined]


def _warn(*args: Any, stacklevel: int = 2, **kwargs: Any) -> None:
    warnings.warn(*args, stacklevel=stacklevel + 1, **kwargs)


def _info(*args: Any, **kwargs: Any) -> None:
    log.info(*args, **kwargs)


def _debug(*args: Any, **kwargs: Any) -> None:
    log.debug(*args, **kwargs)


rank_zero_debug = rank_zero_only(_debug)
rank_zero_info = rank_zero_only(_info)
rank_zero_warn = rank_zero_only(_warn)
_future_warning = partial(warnings.warn, category=FutureWarning)


def _deprecated_root_import_class(name: str, domain: str) -> None:
    """Emit the FutureWarning used by the root-level deprecated aliases."""
    _future_warning(
        f"Importing `{name}` from `torchmetrics_amd` was deprecated and will be removed in 2.0."
        f" Import `{name}` from `torchmetrics_amd.{domain}` instead."
    )


def _deprecated_root_import_func(name: str, domain: str) -> None:
    _future_warning(
        f"Importing `{name}` from `torchmetrics_amd.functional` was deprecated and will be removed in 2.0."
        f" Import `{name}` from `torchmetrics_amd.{domain}` instead."
    )


__all__ = ["rank_zero_only", "rank_zero_debug", "rank_zero_info", "rank_zero_warn"]
