"""Coupling axes — mirror of src/Axes.jl (host-side integer index bookkeeping).

Indices are 1-based like Julia's so that descriptors, summaries and error
messages read exactly as the reference's; the C ABI consumes them as is.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence

__all__ = ["CouplingAxes", "reverse", "is_reverse"]


@dataclass(frozen=True)
class CouplingAxes:
    """``struct CouplingAxes`` — src/Axes.jl:28-35."""

    d: int
    n: int
    axis_id: List[int] = field(default_factory=list)
    axis_af: List[int] = field(default_factory=list)
    axis_nn: List[int] = field(default_factory=list)

    # --- constructors -----------------------------------------------------
    @classmethod
    def from_mask(cls, d: int, mask: Sequence[int], n: int = 0) -> "CouplingAxes":
        """``CouplingAxes(d, mask; n)`` — src/Axes.jl:79-100."""
        mask = [int(m) for m in mask]
        if not mask or max(mask) > d:
            raise AssertionError("The mask cannot contain values higher than the dimension")
        axis_id = [i for i in range(1, d + 1) if i not in mask]      # :88 (sorted)
        axis_af = list(mask)                                          # :91 (given order)
        axis_nn = list(range(1, n + 1)) + [i + n for i in axis_id]    # :98
        return cls(d, n, axis_id, axis_af, axis_nn)

    @classmethod
    def from_cut(cls, d: int, j: int | None = None, n: int = 0, reverse: bool = False) -> "CouplingAxes":
        """``CouplingAxes(d, j=d÷2; n, reverse)`` — src/Axes.jl:104-113."""
        if j is None:
            j = d // 2
        mask = list(range(j + 1, d + 1)) if not reverse else list(range(1, j + 1))
        return cls.from_mask(d, mask, n=n)

    # --- reference semantics ---------------------------------------------
    def __eq__(self, other) -> bool:
        """``==`` — src/Axes.jl:46-56: compares SORTED index sets."""
        if not isinstance(other, CouplingAxes):
            return NotImplemented
        return (self.d == other.d and self.n == other.n and
                sorted(self.axis_id) == sorted(other.axis_id) and
                sorted(self.axis_af) == sorted(other.axis_af) and
                sorted(self.axis_nn) == sorted(other.axis_nn))

    def __hash__(self):
        return hash((self.d, self.n, tuple(sorted(self.axis_id)), tuple(sorted(self.axis_af))))

    def summarize(self) -> str:
        """``summarize(::CouplingAxes)`` — src/Axes.jl:39-43."""
        af = ",".join(str(v) for v in self.axis_af)
        idn = ",".join(str(v) for v in self.axis_id)
        return f"(d,n)=({self.d},{self.n}); identity=({idn}), transformed=({af})"


def CouplingAxes_(d_or_data, mask_or_j=None, n: int = 0, reverse: bool = False) -> CouplingAxes:
    """Julia-style overload resolution of ``CouplingAxes(...)`` (src/Axes.jl:79-119)."""
    from .data import DataArrays  # local import (cycle)

    if isinstance(d_or_data, DataArrays):
        d, n = d_or_data.number_dimensions(), d_or_data.number_conditions()
    else:
        d = int(d_or_data)
    if mask_or_j is None or isinstance(mask_or_j, int):
        return CouplingAxes.from_cut(d, mask_or_j, n=n, reverse=reverse)
    return CouplingAxes.from_mask(d, mask_or_j, n=n)


def reverse(axes: CouplingAxes) -> CouplingAxes:
    """``Base.reverse(axes)`` — src/Axes.jl:129-134."""
    axis_nn = list(range(1, axes.n + 1)) + [i + axes.n for i in axes.axis_af]
    return CouplingAxes(axes.d, axes.n, list(axes.axis_af), list(axes.axis_id), axis_nn)


def is_reverse(a1: CouplingAxes, a2: CouplingAxes) -> bool:
    """``is_reverse`` — src/Axes.jl:137-139 (element-wise, order-sensitive)."""
    return (a1.axis_af == a2.axis_id and a2.axis_af == a1.axis_id and a1.n == a2.n)
