"""GPU parity of the training path (df_train_* through the C ABI) against the
oracle's reverse-mode restatement (oracle/flow_oracle.py: nll_and_grad,
adam_update — pinned by finite differences in tests/test_oracle.py).

Criteria:
  * gradient: fp32 device sums vs the fp64 oracle, per Dense tensor,
    |g - g_ref| <= 1e-4·|g_ref| + 2e-5·max|g_ref| (reductions over the batch
    reorder fp32 sums; the same criterion as helpers.close, looser rtol);
  * Adam: the device update equals the Float32 formula evaluated in numpy
    from the same gradient to 1 ulp;
  * reproducibility: two gradient evaluations are bitwise identical (fixed
    reduction order, no atomics).
"""
import numpy as np
import pytest

import densityflows_amd as dfa
from densityflows_amd.train import Adam, HIPTrainer, load_trainables, setup, train_, trainables
import densityflows_amd.train as train_mod
from helpers import _single_dense_spec, random_net, close, spec_to_element
from oracle import flow_oracle as O

pytestmark = pytest.mark.gpu

G_RTOL = 1e-4
G_ATOL = 2e-5


def _dev(a, dev):
    """numpy (rows, B) → flat Julia-order device buffer."""
    import torch

    a = np.asarray(a, np.float32)
    return torch.from_numpy(np.ascontiguousarray(a.T).ravel()).to(dev)


def _flat_oracle_grads(spec, grads):
    parts = []
    for L, g in zip(O._flat_layers(spec), grads):
        if L["kind"] == "norm":
            continue
        for net in ("s_net", "t_net"):
            if net not in L:
                continue
            for (dW, db), D in zip(g[net], L[net]):
                parts.append(np.asarray(dW).ravel(order="F"))
                if D.get("b") is not None:
                    parts.append(np.asarray(db))
    return np.concatenate(parts)


def _tensor_slices(spec):
    out, o = [], 0
    for L in O._flat_layers(spec):
        if L["kind"] == "norm":
            continue
        for net in ("s_net", "t_net"):
            for D in L.get(net, []):
                out.append(slice(o, o + D["W"].size))
                o += D["W"].size
                if D.get("b") is not None:
                    out.append(slice(o, o + D["b"].size))
                    o += D["b"].size
    return out


def _readme_spec(rng, hidden=16):
    """test/runtests.jl:103-109: three RNVP layers + NormalizationLayer(x, -1, 1)."""
    layers = [O.rnvp_layer(rng, O.coupling_axes(5, m, n=1), hidden=hidden, bias_scale=0.1, out_scale=0.5)
              for m in ([1, 2, 3], [3, 4, 5], [5, 1, 2])]
    layers.append({"kind": "norm", "x_min": np.full(5, -3.0, np.float32), "x_max": np.full(5, 2.5, np.float32),
                   "alpha": -1.0, "beta": 1.0})
    return {"kind": "chain", "layers": layers}


def _cfg2_spec(rng):
    """BASELINE configs[1]: FlowChain(CouplingBlock, 4, 5; hidden 64), n = 0."""
    blocks = []
    for _ in range(4):
        blocks.append(O.coupling_block(rng, O.coupling_axes_cut(5, n=0), hidden=64, bias_scale=0.1,
                                       out_scale=0.1))
    return {"kind": "chain", "layers": blocks}


def _mixed_spec(rng):
    """tanh / sigmoid conditioners, n_sublayers = 1, a NICE layer, hidden 32."""
    nice = O.rnvp_layer(rng, O.coupling_axes(6, [2, 5], n=2), hidden=32, act="tanh", bias_scale=0.1)
    nice["kind"] = "nice"
    del nice["s_net"]
    return {"kind": "chain", "layers": [
        O.rnvp_layer(rng, O.coupling_axes(6, [1, 3, 6], n=2), hidden=32, act="tanh", bias_scale=0.1,
                     out_scale=0.5),
        nice,
        O.coupling_block(rng, O.coupling_axes_cut(6, 2, n=2), n_sub=1, hidden=32, act="sigmoid",
                         bias_scale=0.1, out_scale=0.5),
    ]}


def _wide_spec(rng):
    """hidden 256 (the layer-wise path): a conditioned 8-d chain with MFMA-sized
    outputs (4 transformed dims), a 3-Dense-hidden net and tanh."""
    return {"kind": "chain", "layers": [
        O.coupling_block(rng, O.coupling_axes_cut(8, 4, n=3), hidden=256, bias_scale=0.1, out_scale=0.1),
        O.rnvp_layer(rng, O.coupling_axes(8, [2, 4, 6, 8, 1], n=3), n_sub=3, hidden=128, act="tanh",
                     bias_scale=0.1, out_scale=0.2),
        {"kind": "norm", "x_min": np.full(8, -3.0, np.float32), "x_max": np.full(8, 3.5, np.float32),
         "alpha": 0.0, "beta": 1.0},
    ]}


def _cfg5_spec(rng):
    """BASELINE configs[3]/[4] model: FlowChain(CouplingBlock, 8, 32; n = 8, hidden 256)."""
    return {"kind": "chain", "layers": [
        O.coupling_block(rng, O.coupling_axes_cut(32, n=8), hidden=256, bias_scale=0.1, out_scale=0.1)
        for _ in range(8)]}


SPECS = {"readme": (_readme_spec, 5, 1), "cfg2": (_cfg2_spec, 5, 0), "mixed": (_mixed_spec, 6, 2),
         "wide": (_wide_spec, 8, 3), "cfg5": (_cfg5_spec, 32, 8)}


@pytest.fixture(params=["fused", "layerwise"])
def path(request, monkeypatch):
    """Both training paths: the fused per-net kernel (when the chain takes it) and the
    layer-wise GEMMs, requested through df_train_create_ex (train.DEFAULT_SWEEP is the
    form every HIPTrainer built without an explicit one asks for)."""
    monkeypatch.setattr(train_mod, "DEFAULT_SWEEP",
                        train_mod.SWEEP_LAYERWISE if request.param == "layerwise" else train_mod.SWEEP_AUTO)
    return request.param


def _setup(name, seed=0):
    make, d, n = SPECS[name]
    rng = np.random.default_rng(seed)
    spec = make(rng)
    chain = spec_to_element(spec)
    return spec, chain, d, n


def _inputs(d, n, B, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((d, B)).astype(np.float32)
    th = rng.random((n, B)).astype(np.float32) if n > 0 else np.zeros((0, B), np.float32)
    return x, th


def _gpu_grad(tr, x, th, cuda, n_total=None):
    import torch

    B = x.shape[1]
    lp = torch.zeros(1, dtype=torch.float64, device=cuda)
    tr.gradient(_dev(x, cuda), _dev(th, cuda) if th.shape[0] else None, B, n_total or B, lp)
    torch.cuda.synchronize()
    return tr.grad().detach().cpu().numpy().copy(), float(lp.item())


@pytest.mark.parametrize("name,B", [("readme", 1000), ("cfg2", 3001), ("mixed", 777), ("readme", 1), ("cfg2", 17)])
def test_gradient_parity(cuda, path, name, B):
    spec, chain, d, n = _setup(name)
    tr = HIPTrainer(chain.hip(), Adam())
    np.testing.assert_array_equal(tr.get_params(), trainables(chain))
    x, th = _inputs(d, n, B)
    g, lpsum = _gpu_grad(tr, x, th, cuda)
    loss, ref = O.nll_and_grad(spec, x, th if n else np.zeros((0, B)))
    ref = _flat_oracle_grads(spec, ref)
    assert g.shape == ref.shape
    assert abs(-lpsum / B - loss) <= 1e-5 * max(1.0, abs(loss))
    worst = 0.0
    for sl in _tensor_slices(spec):
        ok, r = close(g[sl], ref[sl], G_RTOL, G_ATOL)
        worst = max(worst, r)
    assert worst <= 1.0, f"gradient violation ratio {worst}"


@pytest.mark.parametrize("name,B", [("cfg2", 3001), ("cfg5", 300), ("wide", 700)])
def test_gradient_parity_exact_f32(cuda, monkeypatch, name, B):
    """The exact-f32 MFMA kernels (DF_F32_EXACT=1: no bf16x3 SPLIT anywhere, DESIGN
    §1b) keep passing the same gradient criterion, and the SPLIT and exact gradients
    agree to it."""
    spec, chain, d, n = _setup(name)
    x, th = _inputs(d, n, B)
    grads = {}
    for exact in ("1", "0"):
        monkeypatch.setenv("DF_F32_EXACT", exact)
        spec, chain, d, n = _setup(name)   # fresh chain and trainer: the plan reads the env
        tr = HIPTrainer(chain.hip(), Adam())
        grads[exact], _ = _gpu_grad(tr, x, th, cuda)
    loss, ref = O.nll_and_grad(spec, x, th if n else np.zeros((0, B)))
    ref = _flat_oracle_grads(spec, ref)
    for sl in _tensor_slices(spec):
        for exact in ("1", "0"):
            ok, r = close(grads[exact][sl], ref[sl], G_RTOL, G_ATOL)
            assert ok, (exact, r)
        assert close(grads["0"][sl], grads["1"][sl], G_RTOL, G_ATOL)[0]


@pytest.mark.parametrize("recompute", [False, True])
@pytest.mark.parametrize("name,B", [("wide", 700), ("wide", 5), ("cfg5", 300)])
def test_gradient_parity_layerwise_wide(cuda, monkeypatch, name, B, recompute):
    """Conditioners beyond the fused kernel (hidden 128/256, 3 hidden Denses, MFMA
    outputs): the layer-wise path is selected automatically.  By default the
    inverse pass keeps the hidden activations (config 5: its features and H1);
    DF_SWEEP_RECOMPUTE recomputes them."""
    monkeypatch.setattr(train_mod, "DEFAULT_SWEEP",
                        train_mod.SWEEP_RECOMPUTE if recompute else train_mod.SWEEP_AUTO)
    test_gradient_parity(cuda, "layerwise", name, B)


@pytest.mark.parametrize("name,B", [("wide", 3001), ("cfg5", 777)])
def test_merged_sweep_bitwise_equals_separate_launches(cuda, monkeypatch, name, B):
    """The merged sweep launches (net i's dW products beside net i+1's output-Dense /
    pullback front, sweep_kernel) compute bitwise the gradient of the separate
    couple_bwd / ldw launches (DF_SWEEP_SEPARATE): same sums in the same order."""
    spec, chain, d, n = _setup(name)
    x, th = _inputs(d, n, B)
    out = []
    for sweep in (train_mod.SWEEP_AUTO, train_mod.SWEEP_LAYERWISE | train_mod.SWEEP_SEPARATE):
        tr = HIPTrainer(spec_to_element(spec).hip(), Adam(), sweep=sweep)
        assert bool(tr.sweep() & train_mod.SWEEP_SEPARATE) == (sweep != train_mod.SWEEP_AUTO)
        out.append(_gpu_grad(tr, x, th, cuda))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


@pytest.mark.parametrize("B", [5, 300, 777, 3001])
def test_h0_free_sweep_bitwise_equals_kept_h0(cuda, B):
    """Config-5 nets (wide SPLIT inverse, relu hidden-256): the default sweep keeps the
    features and H1 only and recomputes H0 inside the split dW1 (with its relu mask for
    the W1ᵀδ1 epilogue).  The recompute is the inverse pass's own first-Dense
    arithmetic, so the gradient and Σ logpdf are bitwise those of the sweep that keeps
    H0 (DF_SWEEP_KEPT); batches below / across the 32-sample dW steps included."""
    spec, chain, d, n = _setup("cfg5")
    x, th = _inputs(d, n, B)
    out = []
    for sweep in (train_mod.SWEEP_AUTO, train_mod.SWEEP_KEPT):
        tr = HIPTrainer(spec_to_element(spec).hip(), Adam(), sweep=sweep)
        want = train_mod.SWEEP_H0FREE if sweep == train_mod.SWEEP_AUTO else train_mod.SWEEP_KEPT
        assert tr.sweep() == want
        out.append(_gpu_grad(tr, x, th, cuda))
        assert tr.sweep() == want  # after the first gradient: the buffers fitted
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def _cfg5_in40_spec(rng):
    """config-5-sized nets whose first Dense takes 40 inputs (d = 32, n = 24): the wide
    SPLIT kernel runs the inverse pass, but the H0-free sweep's 32-float feature rows do
    not hold them."""
    return {"kind": "chain", "layers": [
        O.coupling_block(rng, O.coupling_axes_cut(32, n=24), hidden=256, bias_scale=0.1, out_scale=0.1)
        for _ in range(2)]}


SPECS["cfg5_in40"] = (_cfg5_in40_spec, 32, 24)


@pytest.mark.parametrize("name,sweep,want", [
    ("readme", "AUTO", "FUSED"), ("cfg2", "AUTO", "FUSED"), ("mixed", "AUTO", "FUSED"),
    ("readme", "LAYERWISE", "RECOMPUTE"), ("cfg2", "LAYERWISE", "RECOMPUTE"),
    ("wide", "AUTO", "KEPT"), ("wide", "RECOMPUTE", "RECOMPUTE"),
    ("cfg5", "AUTO", "H0FREE"), ("cfg5", "LAYERWISE", "H0FREE"), ("cfg5", "KEPT", "KEPT"),
    ("cfg5", "RECOMPUTE", "RECOMPUTE"), ("cfg5_in40", "AUTO", "KEPT"),
    ("cfg5", "FUSED", None), ("wide", "H0FREE", None), ("cfg5_in40", "H0FREE", None), ("cfg2", "KEPT", None)])
def test_sweep_form_per_shape(cuda, name, sweep, want):
    """Which reverse sweep each conditioner shape takes (df_train_sweep):
    one production form per shape class, and an explicit request the shape cannot take
    is refused (DF_ERR_UNSUPPORTED) rather than silently served by another form.  The
    form reported before the first gradient is the one the gradient runs (the buffers
    of these batches fit), and the gradient matches the oracle."""
    spec, chain, d, n = _setup(name)
    req = getattr(train_mod, "SWEEP_" + sweep)
    if want is None:
        with pytest.raises(dfa._lib.UnsupportedError):
            HIPTrainer(chain.hip(), Adam(), sweep=req)
        return
    tr = HIPTrainer(chain.hip(), Adam(), sweep=req)
    assert tr.sweep() == getattr(train_mod, "SWEEP_" + want)
    B = 300
    x, th = _inputs(d, n, B)
    g, lpsum = _gpu_grad(tr, x, th, cuda)
    assert tr.sweep() == getattr(train_mod, "SWEEP_" + want)
    loss, ref = O.nll_and_grad(spec, x, th if n else np.zeros((0, B)))
    ref = _flat_oracle_grads(spec, ref)
    assert abs(-lpsum / B - loss) <= 1e-5 * max(1.0, abs(loss))
    for sl in _tensor_slices(spec):
        assert close(g[sl], ref[sl], G_RTOL, G_ATOL)[0]


@pytest.mark.parametrize("name", ["cfg2", "wide"])
def test_gradient_bitwise_reproducible(cuda, path, name):
    spec, chain, d, n = _setup(name)
    tr = HIPTrainer(chain.hip(), Adam())
    x, th = _inputs(d, n, 20000)
    g1, _ = _gpu_grad(tr, x, th, cuda)
    g2, _ = _gpu_grad(tr, x, th, cuda)
    np.testing.assert_array_equal(g1, g2)


def test_gradient_shards_sum(cuda, path):
    """Data-parallel contract: shard gradients with n_total = global batch sum to the full gradient."""
    spec, chain, d, n = _setup("readme")
    tr = HIPTrainer(chain.hip(), Adam())
    x, th = _inputs(d, n, 2000)
    g, _ = _gpu_grad(tr, x, th, cuda)
    ga, _ = _gpu_grad(tr, x[:, :700], th[:, :700], cuda, n_total=2000)
    gb, _ = _gpu_grad(tr, x[:, 700:], th[:, 700:], cuda, n_total=2000)
    for sl in _tensor_slices(spec):
        assert close(ga[sl] + gb[sl], g[sl], 1e-5, 1e-6)[0]


def test_empty_batch_gradient_is_zero(cuda):
    spec, chain, d, n = _setup("readme")
    tr = HIPTrainer(chain.hip(), Adam())
    x, th = _inputs(d, n, 100)
    _gpu_grad(tr, x, th, cuda)
    import torch

    tr.gradient(None, None, 0, 1, None)
    torch.cuda.synchronize()
    assert not np.any(tr.grad().cpu().numpy())


def _ulp_diff(a, b):
    ai = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    bi = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return int(np.max(np.abs(ai - bi))) if ai.size else 0


@pytest.mark.parametrize("name", ["readme", "mixed", "wide"])
def test_adam_step_and_repack(cuda, path, name):
    """Optimisers.update! on the device: the Float32 Adam formula to 1 ulp over
    two steps (βᵗ advances), and the chain's packed weights follow the update
    (forward / backward use the new parameters)."""
    spec, chain, d, n = _setup(name)
    opt = Adam(2e-3, (0.8, 0.99), 1e-7)
    tr = HIPTrainer(chain.hip(), opt)
    p = tr.get_params().copy()
    st = [np.zeros_like(p), np.zeros_like(p), (np.float32(0.8), np.float32(0.99))]
    for step in range(2):
        x, th = _inputs(d, n, 512, seed=10 + step)
        g, _ = _gpu_grad(tr, x, th, cuda)
        p = tr.get_params().copy()
        tr.apply()
        O.adam_update(p, g, st, eta=np.float32(2e-3), beta=(np.float32(0.8), np.float32(0.99)),
                      eps=np.float32(1e-7))
        assert _ulp_diff(tr.get_params(), p) <= 1
    # the chain now evaluates the updated parameters
    load_trainables(chain, tr.get_params())
    x, th = _inputs(d, n, 300, seed=99)
    z, l = dfa.backward(chain, x, th if n else None)
    zo, lo = O.backward(chain.to_spec(), x, th if n else np.zeros((0, 300)))
    assert close(z, zo)[0] and close(l, lo)[0]


def test_set_params_roundtrip(cuda):
    spec, chain, d, n = _setup("readme")
    tr = HIPTrainer(chain.hip(), Adam())
    p = tr.get_params()
    q = (p * np.float32(0.5)).astype(np.float32)
    tr.set_params(q)
    np.testing.assert_array_equal(tr.get_params(), q)
    load_trainables(chain, q)
    x, th = _inputs(d, n, 64, seed=3)
    xf, lf = dfa.forward(chain, x, th)
    xo, lo = O.forward(chain.to_spec(), x, th)
    assert close(xf, xo)[0] and close(lf, lo)[0]


def test_train_runtests_flow(cuda):
    """test/runtests.jl:97-121: datatest.jld2 fixture, README chain, Adam(1f-3),
    train!(epochs = 5), then sample(flow, (2, 5, 7), (-1f0,))."""
    import os

    here = os.path.join(os.path.dirname(__file__), "golden")
    x = np.load(os.path.join(here, "datatest_x.npy"))
    th = np.load(os.path.join(here, "datatest_theta.npy"))
    rng = np.random.default_rng(0)
    data = dfa.DataArrays(x, th, rng=rng)
    chain = dfa.FlowChain(
        dfa.CouplingLayer(data, [1, 2, 3], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.CouplingLayer(data, [3, 4, 5], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.CouplingLayer(data, [5, 1, 2], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.NormalizationLayer.from_data(x, -1.0, 1.0))
    flow = dfa.Flow(chain, data)
    state = setup(Adam(1e-3), flow)
    p0 = trainables(chain)
    x_tr, th_tr = data.training_data()
    l0 = -float(dfa.nll_partial_sum(flow, x_tr, th_tr)[0].item()) / x_tr.shape[1]
    train_(flow, data, state, epochs=5, verbose=False, rng=np.random.default_rng(1))
    assert len(flow.train_loss) == 5 and len(flow.valid_loss) == 5
    assert all(np.isfinite(flow.train_loss)) and all(np.isfinite(flow.valid_loss))
    assert flow.train_loss[-1] < l0
    # the Python model holds the trained parameters (sync_model)
    assert not np.array_equal(trainables(chain), p0)
    x_new = dfa.sample(flow, (2, 5, 7), (-1.0,))
    assert tuple(x_new.shape) == (5, 2, 5, 7)


def test_train_matches_oracle_steps(cuda):
    """Three full train! mini-batch steps (shuffle off) against the oracle's
    gradient + Adam restatement: parameters agree to fp32 tolerance."""
    spec, chain, d, n = _setup("readme", seed=4)
    rng = np.random.default_rng(7)
    x = rng.standard_normal((5, 96)).astype(np.float32)
    th = rng.random((1, 96)).astype(np.float32)
    tr = HIPTrainer(chain.hip(), Adam())
    p = trainables(chain).astype(np.float32)
    st = [np.zeros_like(p), np.zeros_like(p), (np.float32(0.9), np.float32(0.999))]
    ref_spec = chain.to_spec()
    for b0 in range(0, 96, 32):
        xb, tb = x[:, b0:b0 + 32], th[:, b0:b0 + 32]
        import torch

        tr.step(_dev(xb, cuda), _dev(tb, cuda), 32)
        torch.cuda.synchronize()
        _, g = O.nll_and_grad(ref_spec, xb, tb)
        O.adam_update(p, _flat_oracle_grads(ref_spec, g).astype(np.float32), st)
        load_trainables(chain, p)
        ref_spec = chain.to_spec()
    got = tr.get_params()
    # Adam normalises the step (≈ η per coordinate); coordinates whose gradient is
    # near zero can move by O(η) on fp32 noise, so compare at the scale of η.
    assert np.max(np.abs(got - p)) <= 3e-4, np.max(np.abs(got - p))
    assert np.mean(np.abs(got - p)) <= 1e-5


@pytest.mark.parametrize("B", [1000, 17])
def test_gradient_parity_single_dense(cuda, B):
    """Training through single-Dense conditioners (the layer-wise path: the features
    gathered once, the output Dense + coupling pullback, x̄ = Wᵀȳ, dW = ȳ·xᵀ) against
    the FD-pinned oracle gradient."""
    rng = np.random.default_rng(0)
    spec = _single_dense_spec(rng)
    chain = spec_to_element(spec)
    tr = HIPTrainer(chain.hip(), Adam())
    np.testing.assert_array_equal(tr.get_params(), trainables(chain))
    x, th = _inputs(5, 1, B)
    g, lpsum = _gpu_grad(tr, x, th, cuda)
    loss, ref = O.nll_and_grad(spec, x, th)
    ref = _flat_oracle_grads(spec, ref)
    assert g.shape == ref.shape
    assert abs(-lpsum / B - loss) <= 1e-5 * max(1.0, abs(loss))
    for sl in _tensor_slices(spec):
        ok, r = close(g[sl], ref[sl], G_RTOL, G_ATOL)
        assert ok, r


OTHER_ACTS = ["softplus", "logcosh", "leakyrelu", "elu", "swish"]


@pytest.mark.parametrize("act", OTHER_ACTS)
def test_gradient_parity_other_activations(cuda, path, act):
    """Training through softplus / logcosh / leakyrelu / elu / swish conditioners
    (docs/src/documentation.md:99-105 trains a logcosh t-net): σ' by NNlib's
    rules — from the output for leakyrelu / elu, from the kept pre-activation for
    softplus / logcosh / swish — against the finite-difference-pinned oracle
    (tests/test_oracle.py::test_nll_gradient_other_activations_finite_differences)."""
    rng = np.random.default_rng(5)
    spec = {"kind": "chain", "layers": [
        O.rnvp_layer(rng, O.coupling_axes(5, [1, 2, 3], n=1), hidden=16, act=act, bias_scale=0.1, out_scale=0.5),
        O.coupling_block(rng, O.coupling_axes_cut(5, 2, n=1), n_sub=1, hidden=32, act=act, bias_scale=0.1,
                         out_scale=0.5)]}
    _check_grad(cuda, spec, 5, 1, 1500)


def _check_grad(cuda, spec, d, n, B):
    chain = spec_to_element(spec)
    tr = HIPTrainer(chain.hip(), Adam())
    x, th = _inputs(d, n, B)
    g, lpsum = _gpu_grad(tr, x, th, cuda)
    loss, ref = O.nll_and_grad(spec, x, th if n else np.zeros((0, B)))
    ref = _flat_oracle_grads(spec, ref)
    assert abs(-lpsum / B - loss) <= 1e-5 * max(1.0, abs(loss))
    worst = 0.0
    for sl in _tensor_slices(spec):
        worst = max(worst, close(g[sl], ref[sl], G_RTOL, G_ATOL)[1])
    assert worst <= 1.0, f"gradient violation ratio {worst}"


@pytest.mark.parametrize("out_act", ["identity", "softplus", "elu"])
def test_gradient_parity_docs_nets(cuda, out_act):
    """The hand-built conditioners of docs/src/documentation.md:101-104
    (s: Dense(5,32,sigmoid) → Dense(32,16,relu) → Dense(16,4); t: Dense(5,12,relu)
    → Dense(12,16,logcosh) → Dense(16,32,relu) → Dense(32,4)) on an 8-d chain with
    one condition: three hidden Denses select the layer-wise path; the output
    Dense optionally carries an activation of its own."""
    rng = np.random.default_rng(6)
    ax = O.coupling_axes(8, [1, 3, 5, 7], n=1)
    s_net = random_net(rng, [5, 32, 16, 4], ["sigmoid", "relu", out_act])
    t_net = random_net(rng, [5, 12, 16, 32, 4], ["relu", "logcosh", "relu", out_act])
    spec = {"kind": "chain", "layers": [dict(ax, kind="rnvp", s_net=s_net, t_net=t_net),
                                        O.rnvp_layer(rng, O.reverse_axes(ax), hidden=16, act="swish",
                                                     bias_scale=0.1, out_scale=0.5)]}
    _check_grad(cuda, spec, 8, 1, 1200)


def test_data_parallel_train_matches_single(cuda, tmp_path):
    """train! sharded over 2 ranks (gloo, both on GPU 0; RCCL is the same
    all-reduce on a multi-GPU node) follows the single-process run: same
    batches, per-rank gradients with the global mean, summed by all-reduce."""
    import os
    import socket
    import subprocess
    import sys

    import dist_train_worker as W

    p1, tl1, vl1 = W.run()
    out = str(tmp_path / "dp.npz")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(os.path.dirname(__file__), "dist_train_worker.py"), out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    dp = np.load(out)
    np.testing.assert_allclose(dp["train_loss"], tl1, rtol=1e-4)
    np.testing.assert_allclose(dp["valid_loss"], vl1, rtol=1e-4)
    # Adam normalises each step to ≈ η: fp32 reordering of the gradient sums can
    # move near-zero-gradient coordinates by O(η) over the run
    assert np.max(np.abs(dp["params"] - p1)) <= 2e-3
    assert np.mean(np.abs(dp["params"] - p1)) <= 2e-5


def _nice_only_spec(rng):
    layers = []
    for m in ([1, 2], [3, 4], [2, 4]):
        L = O.rnvp_layer(rng, O.coupling_axes(4, m, n=1), hidden=32, bias_scale=0.1)
        L["kind"] = "nice"
        del L["s_net"]
        layers.append(L)
    norm = {"kind": "norm", "x_min": np.full(4, -2.5, np.float32), "x_max": np.full(4, 2.0, np.float32),
            "alpha": -1.0, "beta": 1.0}
    return {"kind": "chain", "layers": [dict(norm), *layers, dict(norm)]}


def _nobias_spec(rng):
    blk = O.coupling_block(rng, O.coupling_axes_cut(6, 3, n=0), hidden=64, bias_scale=0.1, out_scale=0.2)
    for L in (blk["layer_1"], blk["layer_2"]):
        for net in ("s_net", "t_net"):
            L[net][0]["b"] = None          # Dense(...; bias=false)
            L[net][-1]["b"] = None
    return {"kind": "chain", "layers": [blk]}


def _d2_spec(rng):
    return {"kind": "chain", "layers": [
        O.coupling_block(rng, O.coupling_axes_cut(2, 1, n=0), hidden=16, bias_scale=0.1, out_scale=0.5)
        for _ in range(3)]}


SPECS.update({"nice_only": (_nice_only_spec, 4, 1), "nobias": (_nobias_spec, 6, 0), "d2": (_d2_spec, 2, 0)})


@pytest.mark.parametrize("name,B", [("nice_only", 15), ("nice_only", 16), ("nobias", 17), ("nobias", 4097),
                                    ("d2", 33), ("cfg2", 4096)])
def test_gradient_parity_edge_cases(cuda, path, name, B):
    """NICE-only chains between NormalizationLayers, Denses without bias,
    unconditional 2-d chains, and batches around the 16-sample tile."""
    test_gradient_parity(cuda, path, name, B)


@pytest.mark.parametrize("name", ["readme", "cfg2", "mixed", "cfg5"])
def test_step_graph_matches_eager_steps(cuda, path, name):
    """df_train_step_graph (eager on first sight of its buffers, captured on the
    second, replayed after) leaves bitwise the parameters of the same sequence of
    eager df_train_step calls: same kernels, Adam's βᵗ advanced on the device.
    The sequence changes batch size (a new graph), grows the batch past the
    trainer's capacity (buffers reallocated: the old capture is dropped) and
    comes back to the first buffers.  Config 5 runs the H0-free sweep, whose feature
    rows, relu masks and partial rows are reallocated by that growth."""
    import torch

    spec, chain, d, n = _setup(name, seed=7)
    chain2 = spec_to_element(spec)    # a trainer repacks its chain's weights: one chain each
    eager = HIPTrainer(chain.hip(device=cuda.index or 0), Adam(1e-3))
    graph = HIPTrainer(chain2.hip(device=cuda.index or 0), Adam(1e-3))
    seq = (64, 64, 64, 64, 33, 33, 33, 64, 5000, 5000, 5000, 64, 64)
    bufs = {}
    hist = []
    for i, B in enumerate(seq):
        x, th = _inputs(d, n, B, seed=B)
        xd, td = _dev(x, cuda), (_dev(th, cuda) if n else None)
        if B not in bufs:                       # persistent staging buffers per batch size
            bufs[B] = (torch.empty_like(xd), torch.empty_like(td) if n else None)
        xs, ts = bufs[B]
        xs.copy_(xd)
        if n:
            ts.copy_(td)
        eager.step(xd, td, B)
        graph.step_graph(xs, ts, B)
        torch.cuda.synchronize()
        pe, pg = eager.get_params(), graph.get_params()
        hist.append(pe.copy())
        if not np.array_equal(pg, pe):
            # which one is off: replay the sequence up to here on a third, eager trainer
            ref = HIPTrainer(spec_to_element(spec).hip(device=cuda.index or 0), Adam(1e-3))
            for k, Bk in enumerate(seq[:i + 1]):
                xk, tk = _inputs(d, n, Bk, seed=Bk)
                ref.step(_dev(xk, cuda), _dev(tk, cuda) if n else None, Bk)
                torch.cuda.synchronize()
                pr = ref.get_params()
                if not np.array_equal(pr, hist[k]):
                    break
            dif = np.flatnonzero(pg != pe)
            pytest.fail(f"step {i} (B = {B}): graph and eager parameters differ ({dif.size} of {pe.size}, "
                        f"indices {dif.min()}..{dif.max()}, max |diff| {np.abs(pg - pe).max():.3g}); a third eager replay "
                        f"{'matches the eager trainer' if np.array_equal(pr, pe) else 'matches the graph trainer' if np.array_equal(pr, pg) else 'matches neither'}"
                        f" (first eager-vs-eager difference at step {k if not np.array_equal(pr, hist[k]) else None})")


def test_small_kernel_first_normalization_layer_reproducible(cuda, monkeypatch, capfd):
    """Regression (round 6): the two-wave small kernel runs the inverse pass of a chain
    that ends with a NormalizationLayer (the README chain) layer-last-first, so that layer
    is the first it applies.  Both waves write the initial state row; wave 0 then writes
    the normalised row, and without a barrier in between wave 1's initial write could land
    after it and undo it (df_small.hip).  That race made
    test_step_graph_matches_eager_steps[fused-readme] fail in about half of the runs of this
    file (gpurun_out/r06y; none in 5 runs with the barrier, r06aa).  Here: the inverse pass
    (MODE_BWD) and the training gradient (logpdf mode with the per-layer snapshots) at
    B = 5000 (313 workgroups), repeated, must equal the FAST kernel's, bitwise.  (A timing
    race: this test alone did not catch it on the unfixed library in three runs, r06ab.)"""
    import torch

    def run(small):
        monkeypatch.delenv("DF_SMALL_MAX", raising=False)
        if not small:
            monkeypatch.setenv("DF_SMALL_MAX", "0")
        monkeypatch.setenv("DF_DEBUG_LAUNCH", "1")
        spec, chain, d, n = _setup("readme", seed=3)
        B = 5000
        x, th = _inputs(d, n, B, seed=11)
        xt = torch.from_numpy(np.ascontiguousarray(x.T)).to(cuda).T
        tt = torch.from_numpy(np.ascontiguousarray(th.T)).to(cuda).T
        tr = HIPTrainer(chain.hip(), Adam())
        outs = []
        for _ in range(12 if small else 1):
            z, ldj = dfa.backward(chain, xt, tt)
            g, _ = _gpu_grad(tr, x, th, cuda)
            outs.append((z.cpu().numpy().copy(), ldj.cpu().numpy().copy(), g))
        launches = capfd.readouterr().err
        assert ("kernel small " in launches) == small, launches
        monkeypatch.delenv("DF_DEBUG_LAUNCH", raising=False)
        return outs

    ref = run(False)[0]
    for k, out in enumerate(run(True)):
        for what, a, b in zip(("z", "ldj", "gradient"), out, ref):
            assert np.array_equal(a, b), f"repeat {k}: {what} differs from the FAST kernel's"


def test_train_graphs_match_eager(cuda):
    """train_ with the graph-replayed steps (default) equals train_ with eager steps, bitwise."""
    import os

    here = os.path.join(os.path.dirname(__file__), "golden")
    x = np.load(os.path.join(here, "datatest_x.npy"))
    th = np.load(os.path.join(here, "datatest_theta.npy"))
    out = []
    for graphs in (True, False):
        rng = np.random.default_rng(0)
        data = dfa.DataArrays(x, th, rng=rng)
        chain = dfa.FlowChain(
            dfa.CouplingLayer(data, [1, 2, 3], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
            dfa.CouplingLayer(data, [3, 4, 5], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
            dfa.NormalizationLayer.from_data(x, -1.0, 1.0))
        flow = dfa.Flow(chain, data)
        state = setup(Adam(1e-3), flow)
        train_(flow, data, state, epochs=3, batchsize=64, verbose=False, rng=np.random.default_rng(1),
               graphs=graphs)
        out.append((trainables(chain), list(flow.train_loss), list(flow.valid_loss)))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1] and out[0][2] == out[1][2]


# ---------------------------------------------------------------------------
# train!(...; debug) and the epoch loop (src/Flows.jl:380-445)
# ---------------------------------------------------------------------------

def test_debug_refuses_nonfinite_update(cuda):
    """debug = true: a mini-batch with a non-finite loss raises (DF_ERR_NONFINITE)
    and leaves the parameters and the Adam state untouched; without debug the
    update goes through (and poisons the parameters, as in the reference)."""
    import torch

    from densityflows_amd import _lib

    spec, chain, d, n = _setup("readme")
    x, th = _inputs(d, n, 256, seed=5)
    x[2, 17] = np.nan
    tr = HIPTrainer(chain.hip(), Adam())
    p0 = tr.get_params().copy()
    tr.set_debug(True)
    with pytest.raises(_lib.NonFiniteError):
        tr.step(_dev(x, cuda), _dev(th, cuda), 256)
    np.testing.assert_array_equal(tr.get_params(), p0)
    with pytest.raises(_lib.NonFiniteError):        # the graph-replay entry point checks too
        tr.step_graph(_dev(x, cuda), _dev(th, cuda), 256)
    np.testing.assert_array_equal(tr.get_params(), p0)
    xg, _ = _inputs(d, n, 256, seed=6)              # a finite batch still trains
    tr.step(_dev(xg, cuda), _dev(th, cuda), 256)
    assert np.all(np.isfinite(tr.get_params())) and not np.array_equal(tr.get_params(), p0)
    tr.set_debug(False)
    tr.step(_dev(x, cuda), _dev(th, cuda), 256)
    torch.cuda.synchronize()
    assert not np.all(np.isfinite(tr.get_params()))


def _datatest_flow(seed=0):
    import os

    here = os.path.join(os.path.dirname(__file__), "golden")
    x = np.load(os.path.join(here, "datatest_x.npy"))
    th = np.load(os.path.join(here, "datatest_theta.npy"))
    rng = np.random.default_rng(seed)
    data = dfa.DataArrays(x, th, rng=rng)
    chain = dfa.FlowChain(
        dfa.CouplingLayer(data, [1, 2, 3], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.CouplingLayer(data, [3, 4, 5], hidden_dim_s=16, hidden_dim_t=16, σ="tanh", rng=rng),
        dfa.CouplingLayer(data, [5, 1, 2], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.NormalizationLayer.from_data(x, -1.0, 1.0))
    return data, chain, dfa.Flow(chain, data)


def test_train_debug_kwarg(cuda):
    """train_(...; debug=True): NaN in a mini-batch → ArgumentError before its
    update; a clean run returns (nothing, nothing) like the reference."""
    from densityflows_amd import _lib

    data, chain, flow = _datatest_flow()
    state = setup(Adam(1e-3), flow)
    assert train_(flow, data, state, epochs=1, verbose=False, debug=True, shuffle=False) == (None, None)
    data.x = data.x.copy()
    data.x[1, data.partition.training[5]] = np.nan      # first mini-batch (shuffle off)
    p = trainables(chain).copy()
    with pytest.raises(_lib.ArgumentError):
        train_(flow, data, state, epochs=1, verbose=False, debug=True, shuffle=False)
    np.testing.assert_array_equal(state.trainer.get_params(), p)


def test_train_epochs_match_oracle_loop(cuda):
    """Two epochs of train_ (shuffle off, batchsize 64, partial last batch kept)
    against the oracle's epoch loop (nll_and_grad + Adam per mini-batch, then
    the full train / valid losses): the pushed loss vectors agree."""
    data, chain, flow = _datatest_flow(seed=3)
    spec0 = chain.to_spec()
    state = setup(Adam(1e-3), flow)
    train_(flow, data, state, epochs=2, batchsize=64, shuffle=False, verbose=False, graphs=True)
    md = flow.metadata
    x_tr, th_tr = data.training_data()
    x_va, th_va = data.validation_data()
    thn_tr = O.normalize_input(th_tr, md.theta_min, md.theta_max)
    thn_va = O.normalize_input(th_va, md.theta_min, md.theta_max)
    # oracle loop on a fresh copy of the initial parameters
    _, chain_o, _ = _datatest_flow(seed=3)
    p = trainables(chain_o).astype(np.float32)
    st = [np.zeros_like(p), np.zeros_like(p), (np.float32(0.9), np.float32(0.999))]
    spec = spec0
    tl, vl = [], []
    N = x_tr.shape[1]
    for _ in range(2):
        for b0 in range(0, N, 64):
            _, g = O.nll_and_grad(spec, x_tr[:, b0:b0 + 64], thn_tr[:, b0:b0 + 64])
            O.adam_update(p, _flat_oracle_grads(spec, g).astype(np.float32), st)
            load_trainables(chain_o, p)
            spec = chain_o.to_spec()
        tl.append(-float(np.mean(O.flow_logpdf(spec, x_tr, thn_tr, np.float64))))
        vl.append(-float(np.mean(O.flow_logpdf(spec, x_va, thn_va, np.float64))))
    print("train_loss", flow.train_loss, tl, "valid_loss", flow.valid_loss, vl)
    np.testing.assert_allclose(flow.train_loss, tl, rtol=2e-4)
    np.testing.assert_allclose(flow.valid_loss, vl, rtol=2e-4)


def test_graph_step_survives_clock_probe_toggle_and_growth(cuda):
    """the clock-stamp buffer is an eager-launch diagnostic.
    A graph step captured with the probe off, then the probe switched on, the stamp
    buffer grown by a larger eager pass and the graph replayed: the replays match an
    eager twin bitwise, and a capture with the probe on records no stamps (nothing
    is allocated inside the capture)."""
    import torch

    spec, chain, d, n = _setup("readme")
    x, th = _inputs(d, n, 512, seed=21)
    a = HIPTrainer(spec_to_element(spec).hip(), Adam())
    b = HIPTrainer(spec_to_element(spec).hip(), Adam())
    xb, tb = _dev(x, cuda), _dev(th, cuda)
    for _ in range(3):                                   # eager, capture, replay (probe off)
        a.step_graph(xb, tb, 512)
        b.step(xb, tb, 512)
    a.chain.clock_probe(True)
    xl, tl = _inputs(d, n, 1 << 18, seed=22)
    a.chain.apply("backward", xl, tl)                     # eager pass: grows the stamp slots
    torch.cuda.synchronize()
    assert a.chain.clock_read()[2] > 0
    for _ in range(3):                                   # replays of the probe-off capture
        a.step_graph(xb, tb, 512)
        b.step(xb, tb, 512)
    x2, th2 = _inputs(d, n, 300, seed=23)                # a new key captured with the probe on
    xb2, tb2 = _dev(x2, cuda), _dev(th2, cuda)
    for _ in range(3):
        a.step_graph(xb2, tb2, 300)
        b.step(xb2, tb2, 300)
    a.chain.clock_probe(False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.get_params(), b.get_params())
