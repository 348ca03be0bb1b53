"""String enums used for argument parsing (parity: reference ``S/utilities/enums.py:20-154``).

Implemented on the stdlib ``enum`` (no lightning-utilities dependency). Members compare equal to their string value
(case-insensitive), and ``None``-valued members compare equal to ``None``.
"""
from enum import Enum
from typing import Any, List, Optional, Type, TypeVar

_E = TypeVar("_E", bound="EnumStr")


class EnumStr(str, Enum):
    """``str``-valued enum with tolerant lookup."""

    @staticmethod
    def _name() -> str:
        return "Task"

    @classmethod
    def _allowed_matches(cls, source: str = "key") -> List[str]:
        keys = [m.lower() for m in cls._member_names_]
        vals = [str(m.value).lower() if m.value is not None else None for m in cls]
        if source == "key":
            return keys
        if source == "value":
            return vals
        return list(dict.fromkeys(keys + vals))

    @classmethod
    def from_str(cls: Type[_E], value: str, source: str = "key") -> _E:
        """Resolve ``value`` against member names (``source='key'``), values or either."""
        norm = value.replace("-", "_").lower() if isinstance(value, str) else value
        for m in cls:
            if source in ("key", "any") and m.name.lower() == norm:
                return m
            if source in ("value", "any") and m.value is not None and str(m.value).lower() == str(value).lower():
                return m
        raise ValueError(f"Invalid {cls._name()}: expected one of {cls._allowed_matches(source)}, but got {value}.")

    @classmethod
    def try_from_str(cls: Type[_E], value: str, source: str = "key") -> Optional[_E]:
        try:
            return cls.from_str(value, source)
        except ValueError:
            return None

    def __eq__(self, other: Any) -> bool:
        if isinstance(other, Enum):
            other = other.value
        if other is None:
            return self.value == "None"
        return str(self.value).lower() == str(other).lower()

    def __hash__(self) -> int:
        return hash(str(self.value).lower())

    def __str__(self) -> str:
        return str(self.value)


class DataType(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Data type"

    BINARY = "binary"
    MULTILABEL = "multi-label"
    MULTICLASS = "multi-class"
    MULTIDIM_MULTICLASS = "multi-dim multi-class"


class AverageMethod(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Average method"

    MICRO = "micro"
    MACRO = "macro"
    WEIGHTED = "weighted"
    NONE = None
    SAMPLES = "samples"


class MDMCAverageMethod(EnumStr):
    @staticmethod
    def _name() -> str:
        return "MDMC Average method"

    GLOBAL = "global"
    SAMPLEWISE = "samplewise"


class ClassificationTask(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Classification"

    BINARY = "binary"
    MULTICLASS = "multiclass"
    MULTILABEL = "multilabel"


class ClassificationTaskNoBinary(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Classification"

    MULTILABEL = "multilabel"
    MULTICLASS = "multiclass"


class ClassificationTaskNoMultilabel(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Classification"

    BINARY = "binary"
    MULTICLASS = "multiclass"


__all__ = [
    "EnumStr",
    "DataType",
    "AverageMethod",
    "MDMCAverageMethod",
    "ClassificationTask",
    "ClassificationTaskNoBinary",
    "ClassificationTaskNoMultilabel",
]
