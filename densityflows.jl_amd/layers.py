"""Flow elements — mirror of src/Layers.jl, src/affine/*.jl, src/norm/*.jl,
src/Blocks.jl (structure and parameters; evaluation runs in the HIP kernels).

Weights follow Flux exactly: ``Dense.weight`` is (out, in), ``bias`` (out,)
(zeros by default), activations by name (NNlib).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np

from ._lib import ACTIVATIONS, ArgumentError
from .axes import CouplingAxes, CouplingAxes_, is_reverse
from .axes import reverse as reverse_axes

__all__ = ["Dense", "Chain", "FlowElement", "CouplingLayerBase", "RNVPCouplingLayer",
           "NICECouplingLayer", "NormalizationLayer", "CouplingBlock", "CouplingLayer",
           "glorot_uniform", "default_net"]


def glorot_uniform(rng, out_dim: int, in_dim: int) -> np.ndarray:
    """Flux.glorot_uniform for a Dense weight: U(±sqrt(6 / (in + out)))."""
    a = math.sqrt(6.0 / (in_dim + out_dim))
    return ((rng.random((out_dim, in_dim)) * 2.0 - 1.0) * a).astype(np.float32)


class Dense:
    """``Flux.Dense(in => out, σ; bias)``: y = σ.(W*x .+ b)."""

    def __init__(self, W, b=None, act: str = "identity"):
        W = np.asarray(W, dtype=np.float32)
        if W.ndim != 2:
            raise ArgumentError("Dense weight must be a matrix (out, in)")
        if act not in ACTIVATIONS:
            raise ArgumentError(f"unsupported activation {act!r}; supported: {sorted(ACTIVATIONS)}")
        self.W = W
        self.b = None if b is None else np.asarray(b, dtype=np.float32).reshape(-1)
        if self.b is not None and self.b.shape[0] != W.shape[0]:
            raise ArgumentError("bias length must equal the output dimension")
        self.act = act

    @classmethod
    def init(cls, in_dim: int, out_dim: int, act: str = "identity", bias: bool = True, rng=None):
        rng = rng if rng is not None else np.random.default_rng()
        return cls(glorot_uniform(rng, out_dim, in_dim), np.zeros(out_dim, np.float32) if bias else None, act)

    @property
    def in_dim(self) -> int:
        return self.W.shape[1]

    @property
    def out_dim(self) -> int:
        return self.W.shape[0]

    def num_params(self) -> int:
        return self.W.size + (0 if self.b is None else self.b.size)

    def to_spec(self):
        return {"W": self.W, "b": self.b, "act": self.act}


class Chain(list):
    """``Flux.Chain`` of Dense layers (the s / t conditioner)."""

    def __init__(self, layers: Sequence[Dense] = ()):
        super().__init__(layers)
        for k in range(1, len(self)):
            if self[k].in_dim != self[k - 1].out_dim:
                raise ArgumentError(f"Dense {k + 1} expects {self[k].in_dim} inputs but receives {self[k - 1].out_dim}")

    def dims(self) -> List[int]:
        return [self[0].in_dim] + [l.out_dim for l in self]

    def num_params(self) -> int:
        return sum(l.num_params() for l in self)

    def to_spec(self):
        return [l.to_spec() for l in self]


def default_net(input_dim: int, output_dim: int, n: int, hidden_dim: int = 32, act: str = "relu",
                bias: bool = True, rng=None) -> Chain:
    """``_dflt_net`` — src/Layers.jl:33-50:
    Chain(Dense(in, h, σ), (n-1)×Dense(h, h, σ), Dense(h, out, identity))."""
    rng = rng if rng is not None else np.random.default_rng()
    layers = [Dense.init(input_dim, hidden_dim, act, bias, rng)]
    layers += [Dense.init(hidden_dim, hidden_dim, act, bias, rng) for _ in range(n - 1)]
    layers += [Dense.init(hidden_dim, output_dim, "identity", bias, rng)]
    return Chain(layers)


class FlowElement:
    """``abstract type FlowElement`` — src/DensityFlows.jl:45."""

    def __len__(self):
        return 1

    def num_params(self) -> int:
        return 0


class CouplingLayerBase(FlowElement):
    """``abstract type CouplingLayer <: FlowElement`` — src/DensityFlows.jl:48."""

    axes: CouplingAxes


class RNVPCouplingLayer(CouplingLayerBase):
    """``RNVPCouplingLayer(s_net, t_net, axes)`` — src/affine/RNVP.jl:41-48."""

    def __init__(self, s_net: Chain, t_net: Chain, axes: CouplingAxes):
        _check_net(s_net, axes, "s_net")
        _check_net(t_net, axes, "t_net")
        self.s_net, self.t_net, self.axes = Chain(s_net), Chain(t_net), axes

    def num_params(self) -> int:
        return self.s_net.num_params() + self.t_net.num_params()

    def summarize(self) -> str:
        """src/affine/RNVP.jl:59-69."""
        return (f"RNVPCouplingLayer | s_net > {self.s_net.dims()} ({self.s_net.num_params()} parameters)\n"
                f"                  | t_net > {self.t_net.dims()} ({self.t_net.num_params()} parameters)\n"
                f"                  | axes  > {self.axes.summarize()}")

    def to_spec(self):
        return {"kind": "rnvp", "d": self.axes.d, "n": self.axes.n, "axis_id": list(self.axes.axis_id),
                "axis_af": list(self.axes.axis_af), "axis_nn": list(self.axes.axis_nn),
                "s_net": self.s_net.to_spec(), "t_net": self.t_net.to_spec()}


class NICECouplingLayer(CouplingLayerBase):
    """``NICECouplingLayer(t_net, axes)`` — src/affine/NICE.jl:31-36."""

    def __init__(self, t_net: Chain, axes: CouplingAxes):
        _check_net(t_net, axes, "t_net")
        self.t_net, self.axes = Chain(t_net), axes

    def num_params(self) -> int:
        return self.t_net.num_params()

    def summarize(self) -> str:
        return (f"NICECouplingLayer | t_net > {self.t_net.dims()} ({self.t_net.num_params()} parameters)\n"
                f"                  | axes  > {self.axes.summarize()}")

    def to_spec(self):
        return {"kind": "nice", "d": self.axes.d, "n": self.axes.n, "axis_id": list(self.axes.axis_id),
                "axis_af": list(self.axes.axis_af), "axis_nn": list(self.axes.axis_nn),
                "t_net": self.t_net.to_spec()}


def _check_net(net, axes: CouplingAxes, which: str):
    if len(net) == 0:
        raise ArgumentError(f"{which} is empty")
    if net[0].in_dim != len(axes.axis_nn):
        raise AssertionError(f"{which}: input dimension {net[0].in_dim} must equal number of "
                             f"untransformed dimensions + n = {len(axes.axis_nn)}")
    if net[-1].out_dim != len(axes.axis_af):
        raise AssertionError(f"{which}: output dimension {net[-1].out_dim} must equal the number of "
                             f"transformed dimensions {len(axes.axis_af)}")


class NormalizationLayer(FlowElement):
    """``NormalizationLayer(x, α=0, β=1)`` — src/norm/Normalization.jl:30-59."""

    def __init__(self, x_min, x_max, alpha: float = 0.0, beta: float = 1.0):
        self.x_min = np.asarray(x_min, dtype=np.float32).reshape(-1)
        self.x_max = np.asarray(x_max, dtype=np.float32).reshape(-1)
        self.alpha = float(np.float32(alpha))
        self.beta = float(np.float32(beta))
        if not self.beta > self.alpha:
            raise AssertionError("Bounds of the normalisation need to be in the correct order, β > α.")

    @classmethod
    def from_data(cls, x, alpha: float = 0.0, beta: float = 1.0) -> "NormalizationLayer":
        from .data import DataArrays

        if isinstance(x, DataArrays):
            x = x.x
        x = np.asarray(x, dtype=np.float32)
        x2 = x.reshape(x.shape[0], -1)
        return cls(x2.min(axis=1), x2.max(axis=1), alpha, beta)

    def summarize(self) -> str:
        return "Normalization Layer"

    def to_spec(self):
        return {"kind": "norm", "x_min": self.x_min, "x_max": self.x_max,
                "alpha": self.alpha, "beta": self.beta}


class CouplingBlock(FlowElement):
    """``CouplingBlock(layer_1, layer_2)`` — src/Blocks.jl:64-75."""

    def __init__(self, layer_1: CouplingLayerBase, layer_2: CouplingLayerBase):
        if not is_reverse(layer_1.axes, layer_2.axes):
            raise ArgumentError("layer_1 and layer_2 need to have complementary axes")
        self.layer_1, self.layer_2 = layer_1, layer_2

    def __len__(self):
        return 2

    def num_params(self) -> int:
        return self.layer_1.num_params() + self.layer_2.num_params()

    def summarize(self) -> str:
        return self.layer_1.summarize() + "\n" + self.layer_2.summarize()

    def to_spec(self):
        return {"kind": "block", "layer_1": self.layer_1.to_spec(), "layer_2": self.layer_2.to_spec()}

    @classmethod
    def build(cls, *args, layer_type=RNVPCouplingLayer, n: int = 0, reverse: bool = False, rng=None, **kws):
        """``CouplingBlock([T,] d | data | axes, [j | mask]; n, reverse, kws...)`` — src/Blocks.jl:88-120."""
        first = args[0] if args and isinstance(args[0], CouplingAxes) else CouplingAxes_(*args, n=n, reverse=reverse)
        rng = rng if rng is not None else np.random.default_rng()
        l1 = CouplingLayer(layer_type, first, rng=rng, **kws)
        l2 = CouplingLayer(layer_type, reverse_axes(first), rng=rng, **kws)
        return cls(l1, l2)


def CouplingLayer(*args, n: int = 0, reverse: bool = False, n_sublayers_t: int = 2, n_sublayers_s: int = 2,
                  hidden_dim_t: int = 32, hidden_dim_s: int = 32, σ_t: str = "relu", σ_s: str = "relu",
                  hidden_dim: Optional[int] = None, σ: Optional[str] = None, bias: bool = True, rng=None):
    """Julia overloads of ``CouplingLayer(...)`` — src/Layers.jl:110-158.

    ``CouplingLayer([T,] axes | d, [j | mask] | data, [j | mask]; n, reverse, kws...)``
    ``CouplingLayer(t_net, axes)`` → NICE, ``CouplingLayer(s_net, t_net, axes)`` → RNVP.
    ``hidden_dim`` / ``σ`` (the ``kws...`` forwarded to ``_dflt_net``) override the
    per-net values, exactly like the reference's keyword splatting (:129,:132).
    """
    args = list(args)
    # explicit nets
    if args and isinstance(args[0], (Chain, list)) and args[0] and isinstance(args[0][0], Dense):
        if len(args) >= 2 and isinstance(args[1], (Chain, list)) and args[1] and isinstance(args[1][0], Dense):
            axes = args[2] if isinstance(args[2], CouplingAxes) else CouplingAxes_(*args[2:], n=n, reverse=reverse)
            return RNVPCouplingLayer(Chain(args[0]), Chain(args[1]), axes)
        axes = args[1] if isinstance(args[1], CouplingAxes) else CouplingAxes_(*args[1:], n=n, reverse=reverse)
        return NICECouplingLayer(Chain(args[0]), axes)
    layer_type = RNVPCouplingLayer
    if args and isinstance(args[0], type) and issubclass(args[0], CouplingLayerBase):
        layer_type = args.pop(0)
    axes = args[0] if args and isinstance(args[0], CouplingAxes) else CouplingAxes_(*args, n=n, reverse=reverse)
    rng = rng if rng is not None else np.random.default_rng()
    in_dim, out_dim = len(axes.axis_nn), len(axes.axis_af)
    ht = hidden_dim if hidden_dim is not None else hidden_dim_t
    hs = hidden_dim if hidden_dim is not None else hidden_dim_s
    at = σ if σ is not None else σ_t
    as_ = σ if σ is not None else σ_s
    t_net = default_net(in_dim, out_dim, n_sublayers_t, ht, at, bias, rng)   # :129
    if layer_type is NICECouplingLayer:
        return NICECouplingLayer(t_net, axes)                                  # :130
    s_net = default_net(in_dim, out_dim, n_sublayers_s, hs, as_, bias, rng)  # :132
    return RNVPCouplingLayer(s_net, t_net, axes)
