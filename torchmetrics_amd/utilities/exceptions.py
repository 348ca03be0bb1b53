"""Exception / warning types (parity: reference ``S/utilities/exceptions.py:16,20``)."""


class TorchMetricsUserError(Exception):
    """Raised when the user drives the metric lifecycle in an invalid order (e.g. double ``sync``)."""


class TorchMetricsUserWarning(Warning):
    """Warning category for recoverable misuse of a metric."""


__all__ = ["TorchMetricsUserError", "TorchMetricsUserWarning"]
