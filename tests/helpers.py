"""Shared test helpers: convert oracle specs ↔ product objects."""
import numpy as np

import densityflows_amd as dfa
from densityflows_amd.axes import CouplingAxes


def _axes(spec):
    return CouplingAxes(spec["d"], spec["n"], list(spec["axis_id"]), list(spec["axis_af"]), list(spec["axis_nn"]))


def _net(net):
    return dfa.Chain([dfa.Dense(D["W"], D.get("b"), D["act"]) for D in net])


def spec_to_element(spec):
    k = spec["kind"]
    if k == "chain":
        return dfa.FlowChain(*[spec_to_element(e) for e in spec["layers"]])
    if k == "block":
        return dfa.CouplingBlock(spec_to_element(spec["layer_1"]), spec_to_element(spec["layer_2"]))
    if k == "norm":
        return dfa.NormalizationLayer(spec["x_min"], spec["x_max"], spec["alpha"], spec["beta"])
    if k == "rnvp":
        return dfa.RNVPCouplingLayer(_net(spec["s_net"]), _net(spec["t_net"]), _axes(spec))
    if k == "nice":
        return dfa.NICECouplingLayer(_net(spec["t_net"]), _axes(spec))
    raise ValueError(k)


def close(a, b, rtol=1e-5, atol_scale=1e-5):
    """Parity criterion (north_star: 1e-5 relative fp32), with an absolute floor of
    atol_scale × max|expected| so that entries near zero are judged on the scale
    of the array.  Returns (ok, max violation ratio)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    atol = atol_scale * max(1.0, float(np.max(np.abs(b))) if b.size else 1.0)
    tol = atol + rtol * np.abs(b)
    err = np.abs(a - b)
    ratio = float(np.max(err / tol)) if a.size else 0.0
    return ratio <= 1.0, ratio


def _O():
    from oracle import flow_oracle

    return flow_oracle


def random_net(rng, dims, acts, bias_scale=0.1, out_scale=0.5):
    """A Flux.Chain of Dense(dims[i], dims[i+1], acts[i]) (glorot W, U(±bias_scale) b)."""
    net = []
    for i in range(len(dims) - 1):
        W = _O().glorot_uniform(rng, dims[i + 1], dims[i])
        if i == len(dims) - 2:
            W = (W * np.float32(out_scale)).astype(np.float32)
        b = ((rng.random(dims[i + 1]) * 2 - 1) * bias_scale).astype(np.float32)
        net.append({"W": W, "b": b, "act": acts[i]})
    return net


def _single_dense_spec(rng):
    """Conditioners of ONE Dense — Chain(Dense(in, out, σ)), legal in the reference
    (any Flux.Chain is an s/t net, src/affine/RNVP.jl:41-48): identity and tanh RNVP
    nets, a single-Dense NICE net, beside a default two-Dense net, conditioned."""
    ax1 = _O().coupling_axes(5, [3, 4], n=1)
    ax2 = _O().coupling_axes(5, [1, 5, 2], n=1)
    ax3 = _O().coupling_axes(5, [2, 4], n=1)
    n_in = lambda ax: len(ax["axis_nn"])
    l1 = dict(ax1, kind="rnvp", s_net=random_net(rng, [n_in(ax1), 2], ["identity"]),
              t_net=random_net(rng, [n_in(ax1), 2], ["tanh"]))
    l2 = dict(ax2, kind="nice", t_net=random_net(rng, [n_in(ax2), 3], ["identity"]))
    l3 = _O().rnvp_layer(rng, ax3, hidden=16, bias_scale=0.1, out_scale=0.5)
    l3["s_net"] = random_net(rng, [n_in(ax3), 2], ["tanh"])
    return {"kind": "chain", "layers": [l1, l2, l3]}
