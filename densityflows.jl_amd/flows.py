"""Flow / density API — mirror of src/Flows.jl and the @flow_wrapper methods
(src/Macros.jl:104-112): θ is normalised with the Flow's MetaData inside the
fused kernel (df_flow_* entry points).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib
from .chains import FlowChain, _n_of
from .data import DataArrays, MetaData, maximum_theta, minimum_theta
from .hip import as_julia_device, julia_empty

__all__ = ["Flow", "MvNormal", "predict", "sample", "logpdf", "pdf", "training_loss", "validation_loss",
           "nll_partial_sum"]

LOG2PI = float(np.log(2.0 * np.pi))


class MvNormal:
    """Base distribution ``MvNormal(zeros(d), I)`` — src/Flows.jl:114 (the only
    base the fused logpdf supports)."""

    def __init__(self, d: int):
        self.d = d

    def __repr__(self):
        return f"MvNormal(0, I_{self.d})"


class Flow:
    """``Flow([base, ] model, data)`` — src/Flows.jl:37-122."""

    def __init__(self, model: FlowChain, data: Optional[DataArrays] = None, base=None, metadata: MetaData = None,
                 train_loss=None, valid_loss=None):
        if not isinstance(model, FlowChain):
            raise _lib.ArgumentError("Flow needs a FlowChain model")
        if metadata is None:
            if data is None:
                raise _lib.ArgumentError("Flow needs DataArrays (or explicit MetaData)")
            d, n = data.number_dimensions(), data.number_conditions()
            metadata = MetaData("", d, n, np.asarray(minimum_theta(data), np.float32),
                                np.asarray(maximum_theta(data), np.float32))
        self.model = model
        self.metadata = metadata
        self.base = base if base is not None else MvNormal(metadata.d)
        if not isinstance(self.base, MvNormal):
            raise _lib.UnsupportedError("only the standard MvNormal base is fused on device")
        self.train_loss = list(train_loss or [])
        self.valid_loss = list(valid_loss or [])

    @property
    def d(self):
        return self.metadata.d

    @property
    def n(self):
        return self.metadata.n

    def hip(self, device=None):
        h = self.model.hip(device=device, n_hint=self.n)
        if self.n > 0 and h.bounds is None:
            h.set_theta_bounds(self.metadata.theta_min, self.metadata.theta_max)
        return h

    def summarize(self) -> str:
        return ("- model --------------------\n" + self.model.summarize() +
                "\n- base distribution --------\nMvNormal")

    # @flow_wrapper backward forward forward!  (src/DensityFlows.jl:72)
    def forward(self, z, theta=None):
        return self.hip().apply("forward", z, self._theta(theta, z), flow=True)

    def backward(self, x, theta=None):
        return self.hip().apply("backward", x, self._theta(theta, x), flow=True)

    def forward_(self, z, theta=None):
        return self.hip().apply_inplace(z, self._theta(theta, z), flow=True)

    def _theta(self, theta, y):
        if self.n == 0:
            return None
        if theta is None:
            raise _lib.DimensionMismatch("dimensions θ must match (n, dims...) with n number of trained parameters")
        if isinstance(theta, tuple):  # NTuple θ: one condition for every point
            return _broadcast_theta(theta, tuple(y.shape[1:]), y)
        return theta


def _broadcast_theta(theta: tuple, dims, like):
    """``collect(θ) .* ones(T, (1, dims...))`` — src/Flows.jl:182."""
    import torch

    dev = like.device if isinstance(like, torch.Tensor) else torch.device("cuda", torch.cuda.current_device())
    buf, view = julia_empty(len(theta), tuple(dims), dev)
    t = torch.tensor([float(np.float32(v)) for v in theta], dtype=torch.float32, device=dev)
    buf.view(-1, len(theta)).copy_(t.expand(buf.numel() // len(theta), len(theta)))
    if not isinstance(like, torch.Tensor):
        return view.cpu().numpy()
    return view


def predict(flow: Flow, z, theta=None):
    """``predict(flow, z, θ) = forward(flow, z, θ)[1]`` — src/Flows.jl:126."""
    return flow.forward(z, theta)[0]


def sample(flow: Flow, dims: Union[int, Tuple[int, ...]], theta=None, rng=None, seed: Optional[int] = None,
           offset: int = 0):
    """``sample([rng, ] flow, dims [, θ])`` — src/Flows.jl:157-192, one library call
    (``df_flow_sample``): r ~ MvNormal(0, I) drawn on the device from a Philox4x32-10
    stream keyed by ``seed`` (default: 64 bits drawn from ``rng``, a
    ``numpy.random.Generator``, as Julia draws from its ``rng``; Julia's Xoshiro
    stream itself is not reproduced), shape (d, dims...) in Julia memory order,
    then the fused ``forward!`` with θ normalised in the kernel.  θ: an array
    (n, dims...) or an NTuple broadcast to every point (Flows.jl:178-188)."""
    import torch

    if isinstance(dims, int):
        dims = (dims,)
    dims = tuple(int(v) for v in dims)
    if seed is None:
        rng = rng if rng is not None else np.random.default_rng()
        seed = int(rng.integers(0, 2**63 - 1, dtype=np.int64)) * 2 + int(rng.integers(0, 2))
    h = flow.hip()
    dev = h.device
    buf, r = julia_empty(flow.d, dims, dev)
    batch = int(np.prod(dims)) if dims else 1
    thb, bcast = None, False
    if flow.n > 0:
        if theta is None:
            raise AssertionError("dimensions θ must match (n, dims...) with n number of trained parameters")
        if isinstance(theta, tuple):
            if len(theta) != flow.n:
                raise AssertionError("dimensions θ must match (n, dims...) with n number of trained parameters")
            thb = torch.tensor([float(np.float32(v)) for v in theta], dtype=torch.float32, device=dev)
            bcast = True
        else:
            if tuple(theta.shape) != (flow.n,) + dims:
                raise AssertionError("dimensions θ must match (n, dims...) with n number of trained parameters")
            thb, _, _ = as_julia_device(theta, flow.n, dev, "θ")
    h.run_sample(buf, thb, bcast, batch, seed, offset)
    return r


def logpdf(flow: Flow, x, theta=None):
    """``logpdf(flow, x, θ)`` — src/Flows.jl:272-284: backward + base logpdf + ldj (fused)."""
    th = flow._theta(theta, x)
    return flow.hip().logpdf(x, th)


def pdf(flow: Flow, x, theta=None):
    """``pdf = exp.(logpdf)`` — src/Flows.jl:345-349."""
    lp = logpdf(flow, x, theta)
    return np.exp(lp) if isinstance(lp, np.ndarray) else lp.exp()


def nll_partial_sum(flow: Flow, x, theta=None, out=None):
    """Σ_j logpdf(x_j) in fp64 on device (deterministic), plus the sample count —
    the per-rank partial of ``loss`` (src/Flows.jl:352-359)."""
    th = flow._theta(theta, x)
    return flow.hip().logpdf_sum(x, th, out=out)


def training_loss(flow: Flow):
    return flow.train_loss


def validation_loss(flow: Flow):
    return flow.valid_loss
