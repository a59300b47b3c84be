"""Data and metadata — mirror of src/Data.jl (host-side plumbing).

Arrays use the reference's logical Julia shapes ``(d, dims...)`` /
``(n, dims...)``.  The hot path never goes through these helpers: θ
normalisation runs inside the fused kernel (df_flow_* entry points).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

__all__ = ["dflt_theta", "MetaData", "DataPartition", "DataArrays", "normalize_input",
           "resize_output", "minimum_theta", "maximum_theta"]


def dflt_theta(*args, dtype=np.float32):
    """``dflt_θ`` — src/Data.jl:57-65: an empty (0, dims...) array.

    ``dflt_theta(2, 3)`` → shape (0, 2, 3); ``dflt_theta(x)`` → (0, x.shape[1:]...).
    """
    if len(args) == 1 and hasattr(args[0], "shape"):
        x = args[0]
        return np.empty((0,) + tuple(x.shape[1:]), dtype=getattr(x, "dtype", dtype) if isinstance(x, np.ndarray) else dtype)
    if len(args) == 1 and isinstance(args[0], tuple):
        args = args[0]
    return np.empty((0,) + tuple(int(a) for a in args), dtype=dtype)


@dataclass
class MetaData:
    """``MetaData`` — src/Data.jl:75-86."""

    hash: str
    d: int
    n: int
    theta_min: np.ndarray
    theta_max: np.ndarray


def minimum_theta(obj):
    """``minimum_θ`` — src/Data.jl:90,182."""
    if isinstance(obj, MetaData):
        return obj.theta_min
    th = np.asarray(obj.theta)
    return th.reshape(th.shape[0], -1).min(axis=1) if th.size else np.zeros(th.shape[0], np.float32)


def maximum_theta(obj):
    """``maximum_θ`` — src/Data.jl:93,183."""
    if isinstance(obj, MetaData):
        return obj.theta_max
    th = np.asarray(obj.theta)
    return th.reshape(th.shape[0], -1).max(axis=1) if th.size else np.zeros(th.shape[0], np.float32)


@dataclass
class DataPartition:
    """``DataPartition`` — src/Data.jl:96-128 (random train/valid/test split)."""

    training: np.ndarray
    validation: np.ndarray
    testing: np.ndarray

    @classmethod
    def random(cls, n: int, f_training=0.9, f_validation=0.1, rng=None) -> "DataPartition":
        rng = rng if rng is not None else np.random.default_rng()
        p = rng.permutation(n)
        i1 = int(round(n * f_training))
        i2 = i1 + int(round(n * f_validation))
        return cls(p[:i1], p[i1:i2], p[i2:n])


class DataArrays:
    """``DataArrays(x, θ = dflt_θ(x); f_training, f_validation, rng)`` — src/Data.jl:131-170."""

    def __init__(self, x, theta=None, f_training=0.9, f_validation=0.1, rng=None):
        x = np.asarray(x, dtype=np.float32)
        if x.ndim < 2:
            raise AssertionError("data must be an array of size (d, i1, ...) at least")
        theta = dflt_theta(x) if theta is None else np.asarray(theta, dtype=np.float32)
        if tuple(x.shape[1:]) != tuple(theta.shape[1:]):
            raise AssertionError("x and θ must have the same size -- except for the first dimension")
        self.x = x
        self.theta = theta
        self.partition = DataPartition.random(x.shape[1], f_training, f_validation, rng)

    def number_dimensions(self) -> int:
        return self.x.shape[0]

    def number_conditions(self) -> int:
        return self.theta.shape[0]

    def _select(self, idx) -> Tuple[np.ndarray, np.ndarray]:
        return np.take(self.x, idx, axis=1), np.take(self.theta, idx, axis=1)

    def training_data(self):
        return self._select(self.partition.training)

    def validation_data(self):
        return self._select(self.partition.validation)

    def testing_data(self):
        return self._select(self.partition.testing)

    def summarize(self) -> str:
        return (f"Data with size {self.x.shape} and parameters / conditions with size {self.theta.shape}.")


def normalize_input(x, x_min, x_max):
    """``normalize_input`` — src/Data.jl:213-218 (host helper; the kernels fuse it)."""
    x = np.asarray(x, dtype=np.float32)
    lo = np.asarray(x_min, dtype=np.float32).reshape((-1,) + (1,) * (x.ndim - 1))
    hi = np.asarray(x_max, dtype=np.float32).reshape((-1,) + (1,) * (x.ndim - 1))
    diff = hi - lo
    with np.errstate(divide="ignore", invalid="ignore"):
        y = (x - lo) / diff
    y[(diff == 0).reshape(-1), ...] = 0
    return y


def resize_output(y, x_min, x_max):
    """``resize_output`` — src/Data.jl:232."""
    y = np.asarray(y, dtype=np.float32)
    lo = np.asarray(x_min, dtype=np.float32).reshape((-1,) + (1,) * (y.ndim - 1))
    hi = np.asarray(x_max, dtype=np.float32).reshape((-1,) + (1,) * (y.ndim - 1))
    return (hi - lo) * y + lo
