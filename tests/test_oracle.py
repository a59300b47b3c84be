"""Pin the CPU oracle against everything the reference's own tests hold
(test/runtests.jl, doctests) and against the committed golden fixtures.
CPU only."""
import os

import numpy as np
import pytest

import make_golden as G
from helpers import close
from oracle import flow_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# --- test/runtests.jl:33-41 ("axes") ----------------------------------------
def test_axes_equalities():
    a = O.coupling_axes(7, [4, 5, 6, 7], n=2)
    b = O.coupling_axes_cut(7, 3, n=2)
    assert O.axes_equal(a, b)
    # data constructors give the same (d=7, n=2 from the data shape)
    assert O.axes_equal(O.coupling_axes_cut(7, 7 // 2, n=2), b)


def test_axes_mask_order_and_reverse():
    ax = O.coupling_axes(5, [5, 1, 2], n=1)          # Axes.jl:88-98
    assert ax["axis_af"] == [5, 1, 2]                 # user order kept
    assert ax["axis_id"] == [3, 4]                    # sorted complement
    assert ax["axis_nn"] == [1, 4, 5]                 # θ first, then id .+ n
    r = O.reverse_axes(ax)                            # Axes.jl:129-134
    assert r["axis_id"] == [5, 1, 2] and r["axis_af"] == [3, 4]
    assert r["axis_nn"] == [1, 6, 2, 3]               # old af order, unsorted
    assert O.is_reverse(ax, r)


# --- test/runtests.jl:43-64 ("real_NVP") -------------------------------------
@pytest.mark.parametrize("mask", [None, [1, 3, 5, 7]])
def test_rnvp_roundtrip_and_exact_ldj_cancellation(mask):
    rng = np.random.default_rng(0)
    ax = O.coupling_axes_cut(7, 3, n=2) if mask is None else O.coupling_axes(7, mask, n=2)
    layer = O.rnvp_layer(rng, ax)
    z1 = np.full((7, 10), 0.2, np.float32)
    th = np.full((2, 10), 0.1, np.float32)
    x, l1 = O.rnvp_forward(layer, z1, th, np.float32)
    z2, l2 = O.rnvp_backward(layer, x.astype(np.float32), th, np.float32)
    np.testing.assert_allclose(z2, z1, rtol=np.sqrt(np.finfo(np.float32).eps))
    assert np.all(l1 + l2 == 0)       # `.≈ 0f0` with default tolerances ⇒ exact zero


# --- test/runtests.jl:66-95 ("chain") ----------------------------------------
def _runtests_chain(rng):
    l1 = O.rnvp_layer(rng, O.coupling_axes(7, [1, 3, 5, 7], n=2))
    l2 = O.rnvp_layer(rng, O.coupling_axes(7, [4, 2, 5, 1, 6], n=2))
    blk = O.coupling_block(rng, O.coupling_axes(7, [4, 2, 5, 1], n=2))
    x1 = np.full((7, 10), 0.2, np.float32)
    x1[:, 1] = 0.4
    th = np.full((2, 10), 0.1, np.float32)
    th[0, 1] = 0.4
    chain = {"kind": "chain", "layers": [l1, l2, blk, O.normalization_layer(x1)]}
    return chain, x1, th


def test_chain_roundtrip():
    chain, x1, th = _runtests_chain(np.random.default_rng(1))
    z, lb = O.backward(chain, x1, th, np.float32)
    x2, lf = O.forward(chain, z.astype(np.float32), th, np.float32)
    np.testing.assert_allclose(x2, x1, rtol=np.sqrt(np.finfo(np.float32).eps), atol=1e-6)
    assert np.all(np.abs(lf + lb) <= 2e-6)


# --- test/runtests.jl:7-31 ("data") and the datatest.jld2 fixture -----------
def test_normalize_input_range():
    th = np.full((2, 10), 0.1, np.float32)
    th[0, 1] = 0.4
    y = O.normalize_input(th, th.min(axis=1), th.max(axis=1))
    assert y.max() <= 1 and y.min() >= 0
    assert np.all(y[1] == 0)          # max == min row → 0 (Data.jl:216)


def test_datatest_fixture():
    x = np.load(os.path.join(GOLDEN, "datatest_x.npy"))
    th = np.load(os.path.join(GOLDEN, "datatest_theta.npy"))
    assert x.shape == (5, 1000) and x.dtype == np.float32
    assert th.shape == (1, 1000)
    vals, counts = np.unique(th, return_counts=True)
    assert list(vals) == [-1.0, 2.0] and list(counts) == [500, 500]
    nl = O.normalization_layer(x, -1.0, 1.0)
    # backward maps the data range [x_min, x_max] onto [α, β] (Normalization.jl:64-77)
    y, _ = O.norm_backward(nl, x, None, np.float32)
    assert np.allclose(y.min(axis=1), -1, atol=1e-6) and np.allclose(y.max(axis=1), 1, atol=1e-6)


def test_dflt_theta_shapes():
    # Data.jl:47-53 doctests
    assert O.dflt_theta((2, 3)).shape == (0, 2, 3)
    assert O.dflt_theta((4, 5)).shape == (0, 4, 5)


# --- doctests src/Layers.jl:99-104, src/Blocks.jl:51-59 -----------------------
def test_doctest_parameter_counts():
    rng = np.random.default_rng(0)
    ax = O.coupling_axes(3, [1, 3], n=2)
    s = O.default_net(rng, 3, 2, n_sub=1, hidden=10, act="tanh")
    t = O.default_net(rng, 3, 2, n_sub=2, hidden=10, act="tanh")
    assert [l["W"].shape[1] for l in s[:1]] + [l["W"].shape[0] for l in s] == [3, 10, 2]
    assert O.num_params(s) == 62 and O.num_params(t) == 172
    r = O.reverse_axes(ax)
    s2 = O.default_net(rng, len(r["axis_nn"]), len(r["axis_af"]), n_sub=1, hidden=10)
    t2 = O.default_net(rng, len(r["axis_nn"]), len(r["axis_af"]), n_sub=2, hidden=10)
    assert O.num_params(s2) == 61 and O.num_params(t2) == 171


# --- golden fixtures -----------------------------------------------------------
@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_golden_matches_oracle(name):
    spec, g, meta = G.load(name)
    if not meta["weights_stored"]:
        assert G.weights_checksum(spec) == pytest.approx(meta["weights_checksum"], rel=1e-12)
    x, lf = O.forward(spec, g["z"], g["theta"], np.float64)
    np.testing.assert_array_equal(x, g["x_fwd"])
    np.testing.assert_array_equal(lf, g["ldj_fwd"])
    z, lb = O.backward(spec, g["x_in"], g["theta"], np.float64)
    np.testing.assert_array_equal(z, g["z_bwd"])
    np.testing.assert_array_equal(lb, g["ldj_bwd"])
    # invertibility of the fp64 oracle itself
    assert close(g["z_bwd"], g["z"], rtol=1e-5)[0]


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_fp32_oracle_within_parity_tolerance(name):
    """The Flux-like fp32 evaluation meets the 1e-5 criterion vs fp64 — so the
    criterion is attainable by any correct fp32 implementation."""
    spec, g, _ = G.load(name)
    x32, l32 = O.forward(spec, g["z"], g["theta"], np.float32)
    assert close(x32, g["x_fwd"])[0] and close(l32, g["ldj_fwd"])[0]


def test_logpdf_matches_mvnormal():
    rng = np.random.default_rng(3)
    z = rng.standard_normal((5, 7))
    lp = O.mvnormal_logpdf(z, np.float64)
    ref = -0.5 * (5 * np.log(2 * np.pi) + np.sum(z * z, axis=0))
    np.testing.assert_allclose(lp, ref, rtol=1e-14)


# ---------------------------------------------------------------------------
# training restatement (src/Flows.jl:380-445, rrule(RNVP_backward) RNVP.jl:99-147)
# ---------------------------------------------------------------------------

def _grad_chain(rng):
    ax = O.coupling_axes(4, [3, 1], n=1)
    nice = O.rnvp_layer(rng, O.coupling_axes(4, [2, 4], n=1), hidden=8, bias_scale=0.1)
    nice["kind"] = "nice"
    del nice["s_net"]
    return {"kind": "chain", "layers": [
        O.rnvp_layer(rng, ax, hidden=8, bias_scale=0.1),
        O.coupling_block(rng, O.coupling_axes_cut(4, 2, n=1), hidden=8, act="tanh", bias_scale=0.1),
        nice,
        O.rnvp_layer(rng, O.coupling_axes(4, [4], n=1), n_sub=1, hidden=8, act="sigmoid", bias_scale=0.1),
        {"kind": "norm", "x_min": np.array([-2, -1, -3, -1.]), "x_max": np.array([2, 3, 1, 2.]),
         "alpha": -1.0, "beta": 1.0}]}


def test_nll_gradient_matches_finite_differences():
    """The reverse-mode restatement (coupling pullbacks + Dense backprop) is
    pinned by central finite differences of the loss in fp64."""
    rng = np.random.default_rng(0)
    chain = _grad_chain(rng)
    x = rng.standard_normal((4, 7))
    th = rng.random((1, 7))
    loss, grads = O.nll_and_grad(chain, x, th)

    def loss_of():
        z, l = O.backward(chain, x, th)
        return -np.mean(O.mvnormal_logpdf(z) + l)

    assert abs(loss - loss_of()) < 1e-12
    flat = O._flat_layers(chain)
    worst = 0.0
    for li, L in enumerate(flat):
        if L["kind"] == "norm":
            assert grads[li] is None
            continue
        for net in ("s_net", "t_net"):
            if net not in L:
                continue
            for k, D in enumerate(L[net]):
                for key in ("W", "b"):
                    D[key] = D[key].astype(np.float64)
                    for idx in [(0, 0), (D["W"].shape[0] - 1, D["W"].shape[1] - 1)] if key == "W" else [(0,), (-1,)]:
                        orig = D[key][idx]
                        h = 1e-6
                        D[key][idx] = orig + h
                        lp = loss_of()
                        D[key][idx] = orig - h
                        lm = loss_of()
                        D[key][idx] = orig
                        fd = (lp - lm) / (2 * h)
                        g = grads[li][net][k][0 if key == "W" else 1][idx]
                        worst = max(worst, abs(fd - g) / max(1e-6, abs(fd) + abs(g)))
    assert worst < 1e-5, worst


@pytest.mark.parametrize("act", ["softplus", "logcosh", "leakyrelu", "elu", "swish"])
def test_nll_gradient_other_activations_finite_differences(act):
    """NNlib's derivative rules for the activations whose σ' needs the
    pre-activation (softplus, logcosh, swish) or a branch on the output
    (leakyrelu, elu), pinned by central finite differences like the chain above."""
    rng = np.random.default_rng(3)
    chain = {"kind": "chain", "layers": [
        O.rnvp_layer(rng, O.coupling_axes(4, [3, 1], n=1), hidden=8, act=act, bias_scale=0.1),
        O.coupling_block(rng, O.coupling_axes_cut(4, 2, n=1), n_sub=3, hidden=8, act=act, bias_scale=0.1)]}
    x = rng.standard_normal((4, 9))
    th = rng.random((1, 9))
    _, grads = O.nll_and_grad(chain, x, th)

    def loss_of():
        z, l = O.backward(chain, x, th)
        return -np.mean(O.mvnormal_logpdf(z) + l)

    worst = 0.0
    for li, L in enumerate(O._flat_layers(chain)):
        for net in ("s_net", "t_net"):
            for k, D in enumerate(L[net]):
                for key in ("W", "b"):
                    D[key] = D[key].astype(np.float64)
                    idxs = [(0, 0), (D["W"].shape[0] - 1, D["W"].shape[1] - 1), (D["W"].shape[0] // 2, 1)] \
                        if key == "W" else [(0,), (-1,)]
                    for idx in idxs:
                        orig = D[key][idx]
                        h = 1e-5
                        D[key][idx] = orig + h
                        lp = loss_of()
                        D[key][idx] = orig - h
                        lm = loss_of()
                        D[key][idx] = orig
                        fd = (lp - lm) / (2 * h)
                        g = grads[li][net][k][0 if key == "W" else 1][idx]
                        worst = max(worst, abs(fd - g) / max(1e-6, abs(fd) + abs(g)))
    assert worst < 1e-5, worst


def test_nll_gradient_single_dense_conditioners_finite_differences():
    """Conditioners of one Dense (Chain(Dense(in, out, σ)), a legal s/t net in the
    reference, src/affine/RNVP.jl:41-48): every weight and bias of the RNVP and NICE
    single-Dense nets pinned by central finite differences."""
    from helpers import _single_dense_spec

    rng = np.random.default_rng(5)
    chain = _single_dense_spec(rng)
    x = rng.standard_normal((5, 9))
    th = rng.random((1, 9))
    _, grads = O.nll_and_grad(chain, x, th)

    def loss_of():
        z, l = O.backward(chain, x, th)
        return -np.mean(O.mvnormal_logpdf(z) + l)

    worst, checked = 0.0, 0
    for li, L in enumerate(O._flat_layers(chain)):
        for net in ("s_net", "t_net"):
            if net not in L or len(L[net]) != 1:
                continue
            D = L[net][0]
            for key in ("W", "b"):
                D[key] = D[key].astype(np.float64)
                for idx in np.ndindex(D[key].shape):
                    orig = D[key][idx]
                    h = 1e-6
                    D[key][idx] = orig + h
                    lp = loss_of()
                    D[key][idx] = orig - h
                    lm = loss_of()
                    D[key][idx] = orig
                    fd = (lp - lm) / (2 * h)
                    g = grads[li][net][0][0 if key == "W" else 1][idx]
                    worst = max(worst, abs(fd - g) / max(1e-6, abs(fd) + abs(g)))
                    checked += 1
    assert checked > 20 and worst < 1e-5, (checked, worst)


def test_nll_gradient_sums_over_shards():
    """Per-shard gradients with the mean over the global batch sum to the full one."""
    rng = np.random.default_rng(1)
    chain = _grad_chain(rng)
    x = rng.standard_normal((4, 11))
    th = rng.random((1, 11))
    l_all, g_all = O.nll_and_grad(chain, x, th)
    l_a, g_a = O.nll_and_grad(chain, x[:, :5], th[:, :5], n_total=11)
    l_b, g_b = O.nll_and_grad(chain, x[:, 5:], th[:, 5:], n_total=11)
    assert abs(l_all - (l_a + l_b)) < 1e-12
    for ga, gb, gall in zip(g_a, g_b, g_all):
        if gall is None:
            continue
        for net in gall:
            if gall[net] is None:
                continue
            for (wa, ba), (wb, bb), (w, b) in zip(ga[net], gb[net], gall[net]):
                np.testing.assert_allclose(wa + wb, w, rtol=1e-12, atol=1e-14)
                np.testing.assert_allclose(ba + bb, b, rtol=1e-12, atol=1e-14)


def test_adam_matches_published_update():
    """Optimisers.Adam: first step moves every parameter by ≈ η·sign(g)."""
    p = np.array([1.0, -2.0, 3.0], np.float32)
    g = np.array([0.5, -0.25, 1e-3], np.float32)
    st = [np.zeros(3, np.float32), np.zeros(3, np.float32), (np.float32(0.9), np.float32(0.999))]
    O.adam_update(p, g, st, eta=np.float32(1e-3), beta=(np.float32(0.9), np.float32(0.999)),
                  eps=np.float32(1e-8))
    np.testing.assert_allclose(p, [1.0 - 1e-3, -2.0 + 1e-3, 3.0 - 1e-3], rtol=0, atol=2e-6)
    assert st[2][0] == np.float32(0.9) * np.float32(0.9)


# ---------------------------------------------------------------------------
# the C++/OpenMP restatement (oracle/cpu_flow.cpp, bench.py's cpu_baseline)
# ---------------------------------------------------------------------------

def _cpu_flow():
    import os
    import subprocess

    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(here, "oracle", "libcpu_flow.so")):
        subprocess.run(["make", "-C", os.path.join(here, "oracle")], check=True, capture_output=True)
    from oracle import cpu_flow

    return cpu_flow


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_cpu_restatement_matches_oracle(name):
    """The timed CPU proxy computes what the numpy oracle computes: fp64 mode to
    1e-12 of the golden fixtures (made by the fp64 oracle), fp32 mode within the
    fp32 oracle's own distance from them."""
    C = _cpu_flow()
    spec, g, meta = G.load(name)
    d, n = meta["d"], meta["n"]
    th = g["theta"] if n > 0 else np.zeros((0, meta["B"]))
    x, l = C.CPUFlow(spec, d, n, np.float64).forward(g["z"].astype(np.float64), th, threads=4)
    np.testing.assert_allclose(x, g["x_fwd"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(l, g["ldj_fwd"], rtol=1e-12, atol=1e-12)
    x32, l32 = C.CPUFlow(spec, d, n, np.float32).forward(g["z"], th, threads=4)
    xo, lo = O.forward(spec, g["z"], th, np.float32)
    ex = np.max(np.abs(x32 - g["x_fwd"])) / np.max(np.abs(g["x_fwd"]))
    eo = np.max(np.abs(xo - g["x_fwd"])) / np.max(np.abs(g["x_fwd"]))
    assert ex <= max(1e-5, 4 * eo), (ex, eo)


@pytest.mark.parametrize("act", ["tanh", "sigmoid", "softplus", "logcosh", "leakyrelu", "elu", "swish"])
def test_cpu_restatement_layer_zoo(act):
    """NICE, n_sublayers 1/3, a NormalizationLayer and every activation, ragged batch."""
    C = _cpu_flow()
    rng = np.random.default_rng(7)
    nice = O.rnvp_layer(rng, O.coupling_axes(4, [2, 4], n=1), hidden=8, act=act, bias_scale=0.1)
    nice["kind"] = "nice"
    del nice["s_net"]
    spec = {"kind": "chain", "layers": [
        O.rnvp_layer(rng, O.coupling_axes(4, [3, 1], n=1), hidden=8, act=act, bias_scale=0.1),
        O.coupling_block(rng, O.coupling_axes_cut(4, 2, n=1), n_sub=3, hidden=12, act=act, bias_scale=0.1),
        nice,
        O.rnvp_layer(rng, O.coupling_axes(4, [4], n=1), n_sub=1, hidden=8, act=act, bias_scale=0.1),
        {"kind": "norm", "x_min": np.array([-2, -1, -3, -1.]), "x_max": np.array([2, 3, 1, 2.]),
         "alpha": -1.0, "beta": 1.0}]}
    z = rng.standard_normal((4, 301))
    th = rng.random((1, 301))
    x, l = C.CPUFlow(spec, 4, 1, np.float64).forward(z, th, threads=3)
    xo, lo = O.forward(spec, z, th, np.float64)
    np.testing.assert_allclose(x, xo, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(l, lo, rtol=1e-12, atol=1e-12)
