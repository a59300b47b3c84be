"""CPU oracle for the DensityFlows.jl coupling-flow hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``densityflows.jl_amd``)
may import, call or link this module.  It is imported by ``tests/``, by
``__graft_entry__.smoke()`` and by ``bench.py``'s ``cpu_baseline`` leg, and
there only as the checker / the timed CPU proxy.

What it is
----------
A numpy restatement of the reference algorithm (DensityFlows.jl v1.0.0,
``/root/reference``), function by function, each citing the reference
``file:line`` it follows.  Arrays use the reference's *logical* Julia shape
``(d, B)`` (features first, samples second); memory order is irrelevant here.

Two precisions:
  * ``dtype=np.float64``: ground truth for parity checks of the fp32 GPU path.
  * ``dtype=np.float32``: a "Flux-like" unfused fp32 evaluation that follows
    the reference's op sequence (vcat -> gather -> per Dense ``W*x .+ b`` via
    BLAS sgemm -> broadcast activation -> exp -> scatter -> per-layer ldj
    add).  It is also the timed CPU proxy of the (un-runnable) Julia path.

Pinning
-------
Julia / Flux / Distributions are not installable in this pipeline (SURVEY.md
§8c), so the reference cannot be run.  The reference's own tests hold no
numeric golden vectors; the oracle is pinned against every invariant and
fixture they do hold (``tests/test_oracle.py``):
  * ``test/runtests.jl:33-41``  axes equalities,
  * ``test/runtests.jl:43-64``  RNVP round trip and exact ldj cancellation,
  * ``test/runtests.jl:66-95``  chain round trip (mixed chain, unsorted masks,
    NormalizationLayer, |ldj_f + ldj_b| <= 2f-6),
  * ``test/runtests.jl:97-121`` ``datatest.jld2`` fixture + sample shape,
  * doctests ``src/Layers.jl:99-104``, ``src/Blocks.jl:51-59`` (parameter counts),
    ``src/Data.jl:47-53`` (dflt_θ shapes).
Dense / activation / MvNormal numerics come from third-party packages that
are not vendored (Flux >= 0.16.4 / NNlib, Distributions >= 0.25.120); they
are restated from their published definitions and are *parity unpinned*
beyond the invariants above.

Model description (plain dicts, produced by the product's ``to_spec()``)
------------------------------------------------------------------------
  dense  = {"W": (out,in) array, "b": (out,) array or None, "act": str}
  net    = [dense, ...]
  rnvp   = {"kind": "rnvp", "d", "n", "axis_id", "axis_af", "axis_nn",
            "s_net": net, "t_net": net}              (axes are 1-based)
  nice   = {"kind": "nice", ...same axes..., "t_net": net}
  block  = {"kind": "block", "layer_1": layer, "layer_2": layer}
  norm   = {"kind": "norm", "x_min": (d,), "x_max": (d,), "alpha", "beta"}
  chain  = {"kind": "chain", "layers": [element, ...]}
"""
from __future__ import annotations

import math

import numpy as np

LOG2PI = math.log(2.0 * math.pi)

# ----------------------------------------------------------------------------
# Axes  (src/Axes.jl)
# ----------------------------------------------------------------------------


def coupling_axes(d, mask, n=0):
    """``CouplingAxes(d, mask; n)`` — src/Axes.jl:79-100.

    axis_id = sorted complement of mask (:88), axis_af = mask in GIVEN order
    (:91), axis_nn = [1:n ; axis_id .+ n] (:98).  1-based, like Julia."""
    mask = [int(m) for m in mask]
    assert max(mask) <= d, "The mask cannot contain values higher than the dimension"
    axis_id = [i for i in range(1, d + 1) if i not in mask]
    axis_af = list(mask)
    axis_nn = list(range(1, n + 1)) + [i + n for i in axis_id]
    return {"d": d, "n": n, "axis_id": axis_id, "axis_af": axis_af, "axis_nn": axis_nn}


def coupling_axes_cut(d, j=None, n=0, reverse=False):
    """``CouplingAxes(d, j=d÷2; n, reverse)`` — src/Axes.jl:104-113."""
    if j is None:
        j = d // 2
    mask = list(range(j + 1, d + 1)) if not reverse else list(range(1, j + 1))
    return coupling_axes(d, mask, n=n)


def reverse_axes(ax):
    """``Base.reverse(axes)`` — src/Axes.jl:129-134 (swap id/af, nn from old af)."""
    n = ax["n"]
    axis_nn = list(range(1, n + 1)) + [i + n for i in ax["axis_af"]]
    return {"d": ax["d"], "n": n, "axis_id": list(ax["axis_af"]),
            "axis_af": list(ax["axis_id"]), "axis_nn": axis_nn}


def is_reverse(a1, a2):
    """``is_reverse`` — src/Axes.jl:137-139 (element-wise, order-sensitive)."""
    return (len(a1["axis_af"]) == len(a2["axis_id"]) and
            all(x == y for x, y in zip(a1["axis_af"], a2["axis_id"])) and
            len(a2["axis_af"]) == len(a1["axis_id"]) and
            all(x == y for x, y in zip(a2["axis_af"], a1["axis_id"])) and
            a1["n"] == a2["n"])


def axes_equal(x, y):
    """``==(::CouplingAxes, ::CouplingAxes)`` — src/Axes.jl:46-56 (sorted sets)."""
    return (x["d"] == y["d"] and x["n"] == y["n"] and
            sorted(x["axis_id"]) == sorted(y["axis_id"]) and
            sorted(x["axis_af"]) == sorted(y["axis_af"]) and
            sorted(x["axis_nn"]) == sorted(y["axis_nn"]))


# ----------------------------------------------------------------------------
# Activations (NNlib, restated; Flux Dense applies them element-wise)
# ----------------------------------------------------------------------------


def _sigmoid(x):
    # NNlib.sigmoid: t = exp(-|x|); x >= 0 ? 1/(1+t) : t/(1+t)
    t = np.exp(-np.abs(x))
    return np.where(x >= 0, 1 / (1 + t), t / (1 + t)).astype(x.dtype, copy=False)


def _softplus(x):
    # NNlib.softplus: log1p(exp(-|x|)) + relu(x)
    return (np.log1p(np.exp(-np.abs(x))) + np.maximum(x, 0)).astype(x.dtype, copy=False)


# Flux 0.16 ``Dense`` evaluates ``σ = NNlib.fast_act(a.σ, x)`` (Flux
# src/layers/basic.jl, ``(a::Dense)(x)``): for Float32/Float64 arrays tanh is
# replaced by ``tanh_fast`` and σ (sigmoid) by ``sigmoid_fast``.  FAST_ACT
# selects that Flux-faithful evaluation (the default, and what the HIP kernels
# compute); ``set_fast_act(False)`` restores the plain NNlib functions.
FAST_ACT = True

# NNlib.tanh_fast(x::Float32) (NNlib src/activations.jl): a rational
# approximation of tanh(x)/x in x², Horner-evaluated with muladd by evalpoly
# (fused on FMA hardware), |x| with x² >= 66 saturating to sign(x).
_TANH_FAST_N = (1.0, 0.1346604, 0.0035974074, 2.2332108e-5, 1.587199e-8)
_TANH_FAST_D = (1.0, 0.4679937, 0.026262015, 0.0003453992, 8.7767893e-7)


def set_fast_act(on: bool) -> None:
    global FAST_ACT
    FAST_ACT = bool(on)


def _fma(a, b, c):
    """fma in the dtype of ``a``: float32 via an exact float64 product (a·b of two
    float32 is exact in float64; the sum is rounded once more, to float32)."""
    if a.dtype == np.float32:
        return (a.astype(np.float64) * np.float64(b) + np.float64(np.float32(c))).astype(np.float32)
    return a * b + c


def _evalpoly(x2, coeffs):
    dt = x2.dtype.type
    r = np.full_like(x2, dt(coeffs[-1]))
    for c in coeffs[-2::-1]:
        r = _fma(r, x2, dt(c)) if x2.dtype == np.float32 else r * x2 + dt(np.float32(c))
    return r


def tanh_fast(x):
    """NNlib.tanh_fast on Float32 data (coefficients and saturation of the Float32
    method; in float64 mode the same function is evaluated in float64)."""
    dt = x.dtype.type
    x2 = x * x
    n = _evalpoly(x2, _TANH_FAST_N)
    d = _evalpoly(x2, _TANH_FAST_D)
    with np.errstate(invalid="ignore", over="ignore"):
        y = x * (n / d)
    return np.where(x2 < dt(66), y, np.sign(x)).astype(x.dtype, copy=False)


def sigmoid_fast(x):
    """NNlib.sigmoid_fast: sigmoid with ``@fastmath exp`` and the saturations
    x > 40 → 1, x < -80 → 0."""
    dt = x.dtype.type
    y = _sigmoid(x)
    return np.where(x > dt(40), dt(1), np.where(x < dt(-80), dt(0), y)).astype(x.dtype, copy=False)


def activation(name, x):
    """Element-wise activation σ of ``Dense(in, out, σ)`` (Flux / NNlib)."""
    dt = x.dtype.type
    if name == "identity":
        return x
    if name == "relu":
        return np.maximum(x, dt(0))
    if name == "tanh":
        return tanh_fast(x) if FAST_ACT else np.tanh(x)
    if name == "sigmoid":
        return sigmoid_fast(x) if FAST_ACT else _sigmoid(x)
    if name == "softplus":
        return _softplus(x)
    if name == "logcosh":
        # NNlib.logcosh: x + softplus(-2x) - log(2)
        return (x + _softplus(dt(-2) * x) - dt(math.log(2.0))).astype(x.dtype, copy=False)
    if name == "leakyrelu":
        # NNlib.leakyrelu(x, a=0.01) = ifelse(x > 0, x, a*x)
        return np.where(x > 0, x, dt(0.01) * x).astype(x.dtype, copy=False)
    if name == "elu":
        # NNlib.elu(x, α=1) = ifelse(x > 0, x, α*expm1(x))
        return np.where(x > 0, x, np.expm1(x)).astype(x.dtype, copy=False)
    if name == "swish":
        # NNlib.swish(x) = x * sigmoid(x)
        return (x * _sigmoid(x)).astype(x.dtype, copy=False)
    raise ValueError(f"unknown activation {name!r}")


# ----------------------------------------------------------------------------
# Dense / conditioner MLP  (src/Layers.jl:33-50, Flux.Dense: σ.(W*x .+ b))
# ----------------------------------------------------------------------------


def dense(layer, x, dtype):
    W = np.asarray(layer["W"], dtype=dtype)
    y = W @ x
    if layer.get("b") is not None:
        y = y + np.asarray(layer["b"], dtype=dtype)[:, None]
    return activation(layer["act"], y)


def mlp(net, x, dtype):
    for layer in net:
        x = dense(layer, x, dtype)
    return x


def _conditioner_input(layer, y, theta, dtype):
    # input = selectdim(vcat(θ, y), 1, axis_nn)   src/affine/RNVP.jl:157,174,196
    y = np.asarray(y, dtype=dtype)
    th = np.asarray(theta, dtype=dtype).reshape(layer["n"], y.shape[1])
    v = np.concatenate([th, y], axis=0)
    idx = np.asarray(layer["axis_nn"], dtype=np.int64) - 1
    return v[idx, :]


def _ldj_sum(s):
    # ldj = dropdims(sum(s, dims=1), dims=1): accumulate over rows in s order
    # (src/affine/RNVP.jl:180 / :86).  Sequential row order.
    acc = np.zeros(s.shape[1], dtype=s.dtype)
    for k in range(s.shape[0]):
        acc = acc + s[k]
    return acc


# ----------------------------------------------------------------------------
# RealNVP coupling  (src/affine/RNVP.jl)
# ----------------------------------------------------------------------------


def rnvp_forward(layer, z, theta, dtype=np.float64):
    """``forward(::RNVPCouplingLayer, z, θ)`` — src/affine/RNVP.jl:168-187."""
    z = np.asarray(z, dtype=dtype)
    inp = _conditioner_input(layer, z, theta, dtype)
    s = mlp(layer["s_net"], inp, dtype)
    t = mlp(layer["t_net"], inp, dtype)
    ldj = _ldj_sum(s)
    x = z.copy()
    af = np.asarray(layer["axis_af"], dtype=np.int64) - 1
    x[af, :] = z[af, :] * np.exp(s) + t
    return x, ldj


def rnvp_backward(layer, x, theta, dtype=np.float64):
    """``backward(::RNVPCouplingLayer, x, θ)`` — src/affine/RNVP.jl:150-165,
    via ``RNVP_backward`` :77-96: z_af = (x_af - t) .* exp.(-s), ldj = -Σs."""
    x = np.asarray(x, dtype=dtype)
    inp = _conditioner_input(layer, x, theta, dtype)
    s = mlp(layer["s_net"], inp, dtype)
    t = mlp(layer["t_net"], inp, dtype)
    ldj = -_ldj_sum(s)
    z = x.copy()
    af = np.asarray(layer["axis_af"], dtype=np.int64) - 1
    z[af, :] = (x[af, :] - t) * np.exp(-s)
    return z, ldj


def rnvp_forward_inplace(layer, z, theta, dtype=np.float64):
    """``forward!(::RNVPCouplingLayer, z, θ)`` — src/affine/RNVP.jl:190-205."""
    inp = _conditioner_input(layer, z, theta, dtype)
    s = mlp(layer["s_net"], inp, dtype)
    t = mlp(layer["t_net"], inp, dtype)
    af = np.asarray(layer["axis_af"], dtype=np.int64) - 1
    z[af, :] = z[af, :] * np.exp(s) + t
    return None


# ----------------------------------------------------------------------------
# NICE coupling  (src/affine/NICE.jl)
# ----------------------------------------------------------------------------


def nice_forward(layer, z, theta, dtype=np.float64):
    """``forward(::NICECouplingLayer)`` — src/affine/NICE.jl:135-153."""
    z = np.asarray(z, dtype=dtype)
    t = mlp(layer["t_net"], _conditioner_input(layer, z, theta, dtype), dtype)
    x = z.copy()
    af = np.asarray(layer["axis_af"], dtype=np.int64) - 1
    x[af, :] = z[af, :] + t
    return x, np.zeros(z.shape[1], dtype=dtype)


def nice_backward(layer, x, theta, dtype=np.float64):
    """``backward(::NICECouplingLayer)`` — src/affine/NICE.jl:118-132 / :63-81."""
    x = np.asarray(x, dtype=dtype)
    t = mlp(layer["t_net"], _conditioner_input(layer, x, theta, dtype), dtype)
    z = x.copy()
    af = np.asarray(layer["axis_af"], dtype=np.int64) - 1
    z[af, :] = x[af, :] - t
    return z, np.zeros(x.shape[1], dtype=dtype)


def nice_forward_inplace(layer, z, theta, dtype=np.float64):
    """``forward!(::NICECouplingLayer)`` — src/affine/NICE.jl:156-170."""
    t = mlp(layer["t_net"], _conditioner_input(layer, z, theta, dtype), dtype)
    af = np.asarray(layer["axis_af"], dtype=np.int64) - 1
    z[af, :] = z[af, :] + t


# ----------------------------------------------------------------------------
# NormalizationLayer  (src/norm/Normalization.jl)
# ----------------------------------------------------------------------------


def normalization_layer(x, alpha=0.0, beta=1.0, dtype=np.float32):
    """Constructor — src/norm/Normalization.jl:51-57 (per-dim min/max over samples)."""
    x = np.asarray(x, dtype=dtype)
    assert beta > alpha, "Bounds of the normalisation need to be in the correct order, β > α."
    x2 = x.reshape(x.shape[0], -1)
    return {"kind": "norm", "x_min": x2.min(axis=1), "x_max": x2.max(axis=1),
            "alpha": alpha, "beta": beta}


def _norm_ldj_const(layer, dtype):
    xmin = np.asarray(layer["x_min"], dtype=dtype)
    xmax = np.asarray(layer["x_max"], dtype=dtype)
    x_diff = xmax - xmin
    delta = dtype(layer["beta"]) - dtype(layer["alpha"])
    terms = np.log(x_diff / delta)
    acc = terms[0]
    for v in terms[1:]:          # Base.sum over a short vector: sequential
        acc = acc + v
    return acc


def norm_forward(layer, z, theta, dtype=np.float64):
    """``forward(::NormalizationLayer)`` — src/norm/Normalization.jl:79-92:
    x = (x_diff .* z .- α .* x_max .+ β .* x_min) ./ δ,  ldj = +Σ log(x_diff/δ)."""
    z = np.asarray(z, dtype=dtype)
    xmin = np.asarray(layer["x_min"], dtype=dtype)[:, None]
    xmax = np.asarray(layer["x_max"], dtype=dtype)[:, None]
    a, b = dtype(layer["alpha"]), dtype(layer["beta"])
    x_diff = xmax - xmin
    delta = b - a
    x = (x_diff * z - a * xmax + b * xmin) / delta
    ldj = _norm_ldj_const(layer, dtype) * np.ones(z.shape[1], dtype=dtype)
    return x, ldj


def norm_backward(layer, x, theta, dtype=np.float64):
    """``backward(::NormalizationLayer)`` — src/norm/Normalization.jl:64-77:
    z = (β .* (x .- x_min) + α .* (x_max .- x)) ./ x_diff,  ldj = -Σ log(x_diff/δ)."""
    x = np.asarray(x, dtype=dtype)
    xmin = np.asarray(layer["x_min"], dtype=dtype)[:, None]
    xmax = np.asarray(layer["x_max"], dtype=dtype)[:, None]
    a, b = dtype(layer["alpha"]), dtype(layer["beta"])
    x_diff = xmax - xmin
    z = (b * (x - xmin) + a * (xmax - x)) / x_diff
    ldj = -_norm_ldj_const(layer, dtype) * np.ones(x.shape[1], dtype=dtype)
    return z, ldj


def norm_forward_inplace(layer, z, theta, dtype=np.float64):
    """``forward!(::NormalizationLayer)`` — src/norm/Normalization.jl:95-103."""
    x, _ = norm_forward(layer, z, theta, dtype)
    z[...] = x


# ----------------------------------------------------------------------------
# Element dispatch, CouplingBlock, FlowChain
# ----------------------------------------------------------------------------


def forward(elem, z, theta, dtype=np.float64):
    k = elem["kind"]
    if k == "rnvp":
        return rnvp_forward(elem, z, theta, dtype)
    if k == "nice":
        return nice_forward(elem, z, theta, dtype)
    if k == "norm":
        return norm_forward(elem, z, theta, dtype)
    if k == "block":
        # src/Blocks.jl:140-150: layer_1 then layer_2, ldj_1 .+ ldj_2
        y, l1 = forward(elem["layer_1"], z, theta, dtype)
        x, l2 = forward(elem["layer_2"], y, theta, dtype)
        return x, l1 + l2
    if k == "chain":
        # src/Chains.jl:168-184: ldj = ldj_1; ldj = ldj .+ ldj_i (i = 2..n)
        layers = elem["layers"]
        zi, ldj = forward(layers[0], z, theta, dtype)
        for e in layers[1:]:
            zi, li = forward(e, zi, theta, dtype)
            ldj = ldj + li
        return zi, ldj
    raise ValueError(k)


def backward(elem, x, theta, dtype=np.float64):
    k = elem["kind"]
    if k == "rnvp":
        return rnvp_backward(elem, x, theta, dtype)
    if k == "nice":
        return nice_backward(elem, x, theta, dtype)
    if k == "norm":
        return norm_backward(elem, x, theta, dtype)
    if k == "block":
        # src/Blocks.jl:127-137: layer_2 then layer_1, ldj_1 .+ ldj_2
        y, l2 = backward(elem["layer_2"], x, theta, dtype)
        z, l1 = backward(elem["layer_1"], y, theta, dtype)
        return z, l1 + l2
    if k == "chain":
        # src/Chains.jl:149-165: start at chain[end], then chain[n-i+1]
        layers = elem["layers"]
        xi, ldj = backward(layers[-1], x, theta, dtype)
        for e in reversed(layers[:-1]):
            xi, li = backward(e, xi, theta, dtype)
            ldj = ldj + li
        return xi, ldj
    raise ValueError(k)


def forward_inplace(elem, z, theta, dtype=np.float64):
    """``forward!`` — src/Chains.jl:187-197, src/Blocks.jl:153-161."""
    k = elem["kind"]
    if k == "rnvp":
        return rnvp_forward_inplace(elem, z, theta, dtype)
    if k == "nice":
        return nice_forward_inplace(elem, z, theta, dtype)
    if k == "norm":
        return norm_forward_inplace(elem, z, theta, dtype)
    if k == "block":
        forward_inplace(elem["layer_1"], z, theta, dtype)
        forward_inplace(elem["layer_2"], z, theta, dtype)
        return None
    if k == "chain":
        for e in elem["layers"]:
            forward_inplace(e, z, theta, dtype)
        return None
    raise ValueError(k)


# ----------------------------------------------------------------------------
# Flow level: θ normalisation, base density, loss (src/Data.jl, src/Flows.jl)
# ----------------------------------------------------------------------------


def normalize_input(theta, tmin, tmax, dtype=np.float32):
    """``normalize_input`` — src/Data.jl:213-218 (rows with max==min set to 0)."""
    theta = np.asarray(theta, dtype=dtype)
    tmin = np.asarray(tmin, dtype=dtype).reshape(-1, 1)
    tmax = np.asarray(tmax, dtype=dtype).reshape(-1, 1)
    diff = tmax - tmin
    with np.errstate(divide="ignore", invalid="ignore"):
        y = (theta - tmin) / diff
    y[(diff == 0)[:, 0], ...] = 0
    return y


def dflt_theta(shape_tail, dtype=np.float32):  # noqa: D401
    """``dflt_θ`` — src/Data.jl:57-65: an array of shape (0, dims...)."""
    return np.empty((0,) + tuple(shape_tail), dtype=dtype)


def mvnormal_logpdf(z, dtype=np.float64):
    """``logpdf(MvNormal(0, I_d), z)`` — Flows.jl:114,279; Distributions:
    c0 - sqmahal/2 with c0 = -(d*log2π + logdet I)/2."""
    z = np.asarray(z, dtype=dtype)
    d = z.shape[0]
    c0 = -(dtype(d) * dtype(LOG2PI) + dtype(0)) / dtype(2)
    q = np.zeros(z.shape[1], dtype=dtype)
    for i in range(d):
        q = q + z[i] * z[i]
    return c0 - q / dtype(2)


def flow_logpdf(chain, x, theta, dtype=np.float64):
    """``logpdf(flow, x, θ)`` on an already-normalised θ — src/Flows.jl:272-281."""
    z, ldj = backward(chain, x, theta, dtype)
    return mvnormal_logpdf(z, dtype) + ldj


def loss(z, ldj, dtype=np.float64):
    """``loss`` — src/Flows.jl:352-359: -mean(logpdf(base, z) .+ ldj)."""
    return -np.mean(mvnormal_logpdf(z, dtype) + ldj)


# ----------------------------------------------------------------------------
# Model construction helpers used by tests (Layers.jl, Blocks.jl, Chains.jl)
# ----------------------------------------------------------------------------


def glorot_uniform(rng, out_dim, in_dim, dtype=np.float32):
    """Flux.glorot_uniform for a Dense weight (out, in):
    U(-sqrt(6/(in+out)), +sqrt(6/(in+out)))."""
    a = math.sqrt(6.0 / (in_dim + out_dim))
    return ((rng.random((out_dim, in_dim)) * 2.0 - 1.0) * a).astype(dtype)


def default_net(rng, in_dim, out_dim, n_sub=2, hidden=32, act="relu", bias_scale=0.0, out_scale=1.0):
    """``_dflt_net`` — src/Layers.jl:33-50: Dense(in,h,σ), (n-1)×Dense(h,h,σ),
    Dense(h,out,identity).  Zero bias (Flux default) unless bias_scale > 0.
    ``out_scale`` shrinks the final Dense (keeps deep random-init flows finite)."""
    dims = [in_dim] + [hidden] * n_sub + [out_dim]
    acts = [act] * n_sub + ["identity"]
    net = []
    for i in range(len(dims) - 1):
        W = glorot_uniform(rng, dims[i + 1], dims[i])
        if i == len(dims) - 2 and out_scale != 1.0:
            W = (W * np.float32(out_scale)).astype(np.float32)
        b = ((rng.random(dims[i + 1]) * 2 - 1) * bias_scale).astype(np.float32)
        net.append({"W": W, "b": b, "act": acts[i]})
    return net


def rnvp_layer(rng, axes, n_sub=2, hidden=32, act="relu", bias_scale=0.0, out_scale=1.0):
    """``CouplingLayer(RNVPCouplingLayer, axes; ...)`` — src/Layers.jl:113-136."""
    in_dim, out_dim = len(axes["axis_nn"]), len(axes["axis_af"])
    t_net = default_net(rng, in_dim, out_dim, n_sub, hidden, act, bias_scale, out_scale)
    s_net = default_net(rng, in_dim, out_dim, n_sub, hidden, act, bias_scale, out_scale)
    return dict(axes, kind="rnvp", s_net=s_net, t_net=t_net)


def coupling_block(rng, first_axes, **kw):
    """``CouplingBlock(T, first_axes; kws...)`` — src/Blocks.jl:88-102."""
    return {"kind": "block", "layer_1": rnvp_layer(rng, first_axes, **kw),
            "layer_2": rnvp_layer(rng, reverse_axes(first_axes), **kw)}


def num_params(net):
    return sum(l["W"].size + (0 if l.get("b") is None else l["b"].size) for l in net)


# ----------------------------------------------------------------------------
# Training: gradient of the NLL through the inverse pass, Adam
# (src/Flows.jl:380-445, custom pullback src/affine/RNVP.jl:99-147)
# ----------------------------------------------------------------------------

_ACT_GRAD = {
    # derivative of σ expressed through the output y = σ(x) (and x where needed)
    "identity": lambda x, y: np.ones_like(y),
    "relu": lambda x, y: (x > 0).astype(y.dtype),
    "tanh": lambda x, y: 1 - y * y,
    "sigmoid": lambda x, y: y * (1 - y),
    # NNlib's derivative table for the activations Flux broadcasts (NNlib
    # src/activations.jl, UNARY_ACTS; NNlib is not vendored, restated from its
    # published rules): softplus → sigmoid_fast(x), logcosh → tanh(x),
    # leakyrelu → ifelse(Ω > 0, 1, 1//100), elu → deriv_elu(Ω) = ifelse(Ω ≥ 0, 1, Ω + α),
    # swish → Ω + sigmoid_fast(x)·(1 − Ω).  sigmoid_fast is exact sigmoid in fp64.
    "softplus": lambda x, y: _sigmoid(x),
    "logcosh": lambda x, y: np.tanh(x),
    "leakyrelu": lambda x, y: np.where(y > 0, 1.0, 0.01).astype(y.dtype),
    "elu": lambda x, y: np.where(y >= 0, np.ones_like(y), y + 1),
    "swish": lambda x, y: y + _sigmoid(x) * (1 - y),
}


def _mlp_forward_cache(net, x, dtype):
    """Forward through a conditioner keeping (pre, post) activations per Dense."""
    cache = []
    h = x
    for layer in net:
        W = np.asarray(layer["W"], dtype=dtype)
        pre = W @ h
        if layer.get("b") is not None:
            pre = pre + np.asarray(layer["b"], dtype=dtype)[:, None]
        post = activation(layer["act"], pre)
        cache.append((h, pre, post))
        h = post
    return h, cache


def _mlp_backward(net, cache, gout, dtype):
    """Reverse-mode through the Dense chain (Flux/Zygote semantics):
    returns (d input, [(dW, db), ...])."""
    grads = [None] * len(net)
    g = gout
    for k in range(len(net) - 1, -1, -1):
        layer = net[k]
        h, pre, post = cache[k]
        if layer["act"] not in _ACT_GRAD:
            raise NotImplementedError(f"gradient of {layer['act']}")
        d = g * _ACT_GRAD[layer["act"]](pre, post)
        dW = d @ h.T
        db = d.sum(axis=1) if layer.get("b") is not None else None
        grads[k] = (dW, db)
        g = np.asarray(layer["W"], dtype=dtype).T @ d
    return g, grads


def _flat_layers(elem):
    k = elem["kind"]
    if k == "chain":
        out = []
        for e in elem["layers"]:
            out += _flat_layers(e)
        return out
    if k == "block":
        return [elem["layer_1"], elem["layer_2"]]
    return [elem]


def nll_and_grad(chain, x, theta, n_total=None, dtype=np.float64):
    """loss = -mean(logpdf(base, z) .+ ldj) with (z, ldj) = backward(chain, x, θ)
    (src/Flows.jl:352-359, :400-413) and its gradient w.r.t. every Dense weight
    and bias.  The mean is over ``n_total`` samples (default: x.shape[1]) so that
    shard gradients sum to the global one.  Returns (loss_sum_part, grads) where
    grads mirrors the flattened layer list: for each coupling layer a dict
    {"s_net": [(dW, db), ...], "t_net": [...]} (None for NormalizationLayer)."""
    layers = _flat_layers(chain)
    B = x.shape[1]
    N = float(n_total if n_total is not None else B)
    u = np.asarray(x, dtype=dtype)
    th = np.asarray(theta, dtype=dtype).reshape(-1, B)
    saved = []
    ldj = np.zeros(B, dtype=dtype)
    # inverse pass, last layer first (src/Chains.jl:149-165)
    for L in reversed(layers):
        k = L["kind"]
        if k == "norm":
            saved.append((L, u, None))
            u, l = norm_backward(L, u, th, dtype)
            ldj = ldj + l
            continue
        inp = _conditioner_input(L, u, th, dtype)
        t, tcache = _mlp_forward_cache(L["t_net"], inp, dtype)
        if k == "rnvp":
            s, scache = _mlp_forward_cache(L["s_net"], inp, dtype)
        else:
            s, scache = np.zeros_like(t), None
        af = np.asarray(L["axis_af"], dtype=np.int64) - 1
        z = u.copy()
        z[af, :] = (u[af, :] - t) * np.exp(-s)
        saved.append((L, u, (inp, s, t, scache, tcache, af, z)))
        if k == "rnvp":
            ldj = ldj - _ldj_sum(s)
        u = z
    z = u
    lp = mvnormal_logpdf(z, dtype) + ldj
    loss_part = -np.sum(lp) / N
    # reverse mode: d loss / d z = z / N ; d loss / d ldj = -1/N
    zbar = z / N
    jbar = -1.0 / N
    grads = []
    for L, u_in, extra in reversed(saved):
        if L["kind"] == "norm":
            xmin = np.asarray(L["x_min"], dtype=dtype)[:, None]
            xmax = np.asarray(L["x_max"], dtype=dtype)[:, None]
            zbar = zbar * (dtype(L["beta"]) - dtype(L["alpha"])) / (xmax - xmin)
            grads.append(None)
            continue
        inp, s, t, scache, tcache, af, z = extra
        e = np.exp(-s)
        zbar_af = zbar[af, :]
        # rrule(RNVP_backward), src/affine/RNVP.jl:119-143
        sbar = -zbar_af * (u_in[af, :] - t) * e - jbar
        tbar = -zbar_af * e
        ubar = zbar.copy()
        ubar[af, :] = zbar_af * e
        g_in_t, gt = _mlp_backward(L["t_net"], tcache, tbar, dtype)
        g_in = g_in_t
        gs = None
        if L["kind"] == "rnvp":
            g_in_s, gs = _mlp_backward(L["s_net"], scache, sbar, dtype)
            g_in = g_in + g_in_s
        else:
            # NICE_backward pullback (src/affine/NICE.jl:102-111): t̄ = -z̄_af, ū = z̄
            pass
        # scatter the conditioner-input gradient back to the state rows
        # (vcat(θ, u)[axis_nn]; θ gets no gradient that we keep)
        nn = np.asarray(L["axis_nn"], dtype=np.int64) - 1
        n = L["n"]
        for kk, slot in enumerate(nn):
            if slot >= n:
                ubar[slot - n, :] += g_in[kk, :]
        zbar = ubar
        grads.append({"s_net": gs, "t_net": gt})
    # reversed(saved) visits layers in chain order, so grads already is
    return loss_part, grads


def adam_update(params, grads, state, eta=1e-3, beta=(0.9, 0.999), eps=1e-8):
    """Optimisers.Adam (v0.4) on flat float arrays, in place:
    m = β1 m + (1-β1) g;  v = β2 v + (1-β2) g²;
    x -= η · (m / (1-β1^t)) / (sqrt(v / (1-β2^t)) + ϵ)."""
    T = params.dtype.type  # Optimisers: η, β, ϵ converted to the parameter eltype
    eta, beta, eps = T(eta), (T(beta[0]), T(beta[1])), T(eps)
    m, v, bt = state
    m[:] = beta[0] * m + (1 - beta[0]) * grads
    v[:] = beta[1] * v + (1 - beta[1]) * (grads * grads)  # (1 - β2) * abs2(dx)
    upd = m / (1 - bt[0]) / (np.sqrt(v / (1 - bt[1])) + eps) * eta
    params -= upd
    state[2] = (bt[0] * beta[0], bt[1] * beta[1])
    return params
