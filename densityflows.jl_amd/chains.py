"""FlowChain and the generic ``forward`` / ``backward`` / ``forward!`` —
mirror of src/Chains.jl.  Every evaluation goes through the fused HIP kernels
(one launch per call for the whole chain); there is no CPU path.
"""
from __future__ import annotations

from typing import Sequence

from . import _lib
from .layers import FlowElement

__all__ = ["FlowChain", "concatenate", "forward", "backward", "forward_", "forward_inplace"]


class FlowChain(FlowElement):
    """``FlowChain(elements...)`` — src/Chains.jl:78-101."""

    def __init__(self, *elements):
        if len(elements) == 1 and isinstance(elements[0], (tuple, list)):
            elements = tuple(elements[0])
        for e in elements:
            if not isinstance(e, FlowElement):
                raise _lib.ArgumentError(f"{type(e).__name__} is not a FlowElement")
        self.layers = tuple(elements)
        self._hip = {}

    @classmethod
    def repeat(cls, element_type, count: int, *args, **kws) -> "FlowChain":
        """``FlowChain([T = CouplingBlock, ], n, args...; kws...)`` — src/Chains.jl:100-101."""
        from .layers import CouplingBlock

        if element_type is CouplingBlock:
            return cls(*[CouplingBlock.build(*args, **kws) for _ in range(count)])
        return cls(*[element_type(*args, **kws) for _ in range(count)])

    # Base.getindex / length / first / last / iterate — src/Chains.jl:125-138
    def __len__(self):
        return len(self.layers)

    def __getitem__(self, i):
        return self.layers[i]

    def __iter__(self):
        return iter(self.layers)

    def num_params(self) -> int:
        return sum(e.num_params() for e in self.layers)

    def summarize(self) -> str:
        return "\n".join(e.summarize() for e in self.layers)

    def to_spec(self):
        return {"kind": "chain", "layers": [e.to_spec() for e in self.layers]}

    def invalidate(self):
        """Drop compiled device handles (call after changing weights in place)."""
        self._hip.clear()

    def hip(self, device=None, n_hint=None):
        from .hip import HIPChain, _torch

        torch = _torch()
        if not torch.cuda.is_available():
            raise _lib.HIPError("no HIP device visible: the fused kernels need an MI355X (gfx950)")
        dev = torch.cuda.current_device() if device is None else torch.device(device).index or 0
        key = (dev, n_hint)
        h = self._hip.get(key)
        if h is None:
            h = HIPChain(self.layers, device=dev, n_hint=n_hint)
            self._hip[key] = h
        return h


def concatenate(*xs) -> FlowChain:
    """``concatenate`` — src/Chains.jl:112-123."""
    if len(xs) == 1 and isinstance(xs[0], tuple):
        xs = xs[0]
    layers = []
    for x in xs:
        if isinstance(x, FlowChain):
            layers += list(x.layers)
        elif isinstance(x, tuple):
            layers += list(x)
        else:
            layers.append(x)
    return FlowChain(*layers)


def _as_chain(elem) -> FlowChain:
    if isinstance(elem, FlowChain):
        return elem
    cached = getattr(elem, "_as_chain", None)
    if cached is None:
        cached = FlowChain(elem)
        elem._as_chain = cached
    return cached


def _n_of(theta):
    return None if theta is None else int(theta.shape[0])


def forward(elem, z, theta=None):
    """``forward(f, z [, θ = dflt_θ(z)])`` → (x, ldj) — src/Chains.jl:168-184 (and per element)."""
    ch = _as_chain(elem)
    return ch.hip(n_hint=_n_of(theta)).apply("forward", z, theta)


def backward(elem, x, theta=None):
    """``backward(f, x [, θ = dflt_θ(x)])`` → (z, ldj) — src/Chains.jl:149-165."""
    ch = _as_chain(elem)
    return ch.hip(n_hint=_n_of(theta)).apply("backward", x, theta)


def forward_(elem, z, theta=None):
    """``forward!(f, z [, θ])`` — src/Chains.jl:187-197: z is transformed in place."""
    ch = _as_chain(elem)
    return ch.hip(n_hint=_n_of(theta)).apply_inplace(z, theta)


forward_inplace = forward_
