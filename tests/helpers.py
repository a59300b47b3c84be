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
