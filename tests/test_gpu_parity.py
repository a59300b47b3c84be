"""GPU parity: the fused HIP path (through the C ABI) against the CPU oracle
and the committed golden fixtures.

Criterion (BASELINE.json north_star): 1e-5 relative fp32 tolerance, with an
absolute floor of 1e-5 × max|expected| (helpers.close); bit-exact for
index/mask selection (identity dims are copied, never recomputed) and exact
forward/inverse ldj cancellation per layer (test/runtests.jl:54,62).
"""
import numpy as np
import pytest

import densityflows_amd as dfa
import make_golden as G
from helpers import close, spec_to_element
from oracle import flow_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _t(a, dev):
    """numpy (rows, B) → Julia-layout (column-major) device tensor."""
    import torch

    a = np.asarray(a, np.float32)
    return torch.from_numpy(np.ascontiguousarray(a.T)).to(dev).T


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_golden_forward_backward(cuda, name):
    spec, g, meta = G.load(name)
    chain = spec_to_element(spec)
    th = _t(g["theta"], cuda) if meta["n"] > 0 else None
    x, lf = dfa.forward(chain, _t(g["z"], cuda), th)
    ok, r = close(_np(x), g["x_fwd"], RTOL)
    assert ok, f"forward x ratio {r}"
    ok, r = close(_np(lf), g["ldj_fwd"], RTOL)
    assert ok, f"forward ldj ratio {r}"
    z, lb = dfa.backward(chain, _t(g["x_in"], cuda), th)
    ok, r = close(_np(z), g["z_bwd"], RTOL)
    assert ok, f"backward z ratio {r}"
    ok, r = close(_np(lb), g["ldj_bwd"], RTOL)
    assert ok, f"backward ldj ratio {r}"


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_identity_dims_bit_exact(cuda, name):
    """Dims a layer does not transform are copied bit for bit: with a single
    coupling layer the identity rows of x equal z exactly."""
    spec, g, meta = G.load(name)
    first = spec["layers"][0]
    layer = first["layer_1"] if first["kind"] == "block" else first
    el = spec_to_element(layer)
    th = _t(g["theta"], cuda) if meta["n"] > 0 else None
    x, _ = dfa.forward(el, _t(g["z"], cuda), th)
    idx = np.asarray(layer["axis_id"]) - 1
    np.testing.assert_array_equal(_np(x)[idx], g["z"][idx])


@pytest.mark.parametrize("mask", [None, [1, 3, 5, 7], [4, 2, 5, 1, 6]])
def test_runtests_real_nvp(cuda, mask):
    """test/runtests.jl:43-64 on the GPU path: round trip and EXACT ldj cancellation."""
    rng = np.random.default_rng(5)
    layer = (dfa.CouplingLayer(dfa.RNVPCouplingLayer, 7, 3, n=2, rng=rng) if mask is None
             else dfa.CouplingLayer(dfa.RNVPCouplingLayer, 7, mask, n=2, rng=rng))
    z1 = np.full((7, 10), 0.2, np.float32)
    th = np.full((2, 10), 0.1, np.float32)
    x, l1 = dfa.forward(layer, _t(z1, cuda), _t(th, cuda))
    z2, l2 = dfa.backward(layer, x, _t(th, cuda))
    np.testing.assert_allclose(_np(z2), z1, rtol=np.sqrt(np.finfo(np.float32).eps))
    assert np.all(_np(l1) + _np(l2) == 0)
    # and against the oracle
    xo, lo = O.forward(layer.to_spec(), z1, th, np.float64)
    assert close(_np(x), xo, RTOL)[0] and close(_np(l1), lo, RTOL)[0]


def test_runtests_chain(cuda):
    """test/runtests.jl:66-95: mixed chain (unsorted masks, block, NormalizationLayer)."""
    rng = np.random.default_rng(6)
    layer_1 = dfa.CouplingLayer(dfa.RNVPCouplingLayer, 7, [1, 3, 5, 7], n=2, rng=rng)
    layer_2 = dfa.CouplingLayer(dfa.RNVPCouplingLayer, 7, [4, 2, 5, 1, 6], n=2, rng=rng)
    block = dfa.CouplingBlock.build(7, [4, 2, 5, 1], n=2, rng=rng)
    small = dfa.FlowChain(layer_1, layer_2)
    assert len(dfa.concatenate(small, block)) == 3
    assert len(dfa.concatenate(block, small)) == 3
    x1 = np.full((7, 10), 0.2, np.float32)
    th = np.full((2, 10), 0.1, np.float32)
    x1[:, 1] = 0.4
    th[0, 1] = 0.4
    chain = dfa.concatenate((small, dfa.FlowChain(block, dfa.NormalizationLayer.from_data(x1))))
    assert isinstance(chain[-1], dfa.NormalizationLayer)
    z, lb = dfa.backward(chain, _t(x1, cuda), _t(th, cuda))
    x2, lf = dfa.forward(chain, z, _t(th, cuda))
    np.testing.assert_allclose(_np(x2), x1, rtol=np.sqrt(np.finfo(np.float32).eps), atol=1e-6)
    assert np.all(np.abs(_np(lf) + _np(lb)) <= 2e-6)
    zo, lbo = O.backward(chain.to_spec(), x1, th, np.float64)
    assert close(_np(z), zo, RTOL)[0] and close(_np(lb), lbo, RTOL)[0]


@pytest.mark.parametrize("name", ["cfg1", "cfg2"])
def test_flow_level_theta_normalisation_and_logpdf(cuda, name):
    """@flow_wrapper (θ normalised in-kernel) and fused logpdf / logpdf_sum."""
    spec, g, meta = G.load(name)
    chain = spec_to_element(spec)
    md = dfa.MetaData("", meta["d"], meta["n"], g["theta_min"], g["theta_max"])
    flow = dfa.Flow(chain, metadata=md)
    th_raw = _t(g["theta_raw"], cuda) if meta["n"] > 0 else None
    x, lf = flow.forward(_t(g["z"], cuda), th_raw)
    assert close(_np(x), g["x_fwd"], RTOL)[0] and close(_np(lf), g["ldj_fwd"], RTOL)[0]
    lp = dfa.logpdf(flow, _t(g["x_in"], cuda), th_raw)
    ok, r = close(_np(lp), g["logpdf"], RTOL)
    assert ok, r
    s, cnt = dfa.nll_partial_sum(flow, _t(g["x_in"], cuda), th_raw)
    assert cnt == meta["B"]
    assert abs(float(s.item()) - float(np.sum(_np(lp).astype(np.float64)))) <= 1e-9 * meta["B"] * 10
    assert abs(float(s.item()) - float(np.sum(g["logpdf"]))) <= 1e-5 * np.sum(np.abs(g["logpdf"]))


def test_forward_inplace_matches_forward(cuda):
    spec, g, _ = G.load("cfg2")
    chain = spec_to_element(spec)
    x, _ = dfa.forward(chain, _t(g["z"], cuda))
    zz = _t(g["z"], cuda)
    dfa.forward_(chain, zz)
    np.testing.assert_array_equal(_np(zz), _np(x))


@pytest.mark.parametrize("name", ["cfg1", "cfg2"])
def test_folded_bias_bit_identical(cuda, name, monkeypatch):
    """The specialised kernel's FAST variant folds the first Dense's bias into the
    last k-slot of the MFMA chain (df_plan.cpp pass 1c): fma(b, 1, W*x) rounds
    exactly like the separate `W*x .+ b`, so x, ldj and the inverse are bitwise
    those of the unfolded plan (DF_NO_FOLD=1) and of the non-FAST variant.  All three
    on exact-f32 MFMA (DF_F32_EXACT=1: the SPLIT variant rounds differently, see
    test_split_variant_accuracy)."""
    spec, g, meta = G.load(name)
    th = _t(g["theta"], cuda) if meta["n"] > 0 else None
    monkeypatch.setenv("DF_F32_EXACT", "1")
    outs = []
    for env in ({}, {"DF_NO_FAST": "1"}, {"DF_NO_FOLD": "1"}):
        for k in ("DF_NO_FAST", "DF_NO_FOLD"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        chain = spec_to_element(spec)       # fresh handle: the plan reads the env at creation
        x, lf = dfa.forward(chain, _t(g["z"], cuda), th)
        z, lb = dfa.backward(chain, _t(g["x_in"], cuda), th)
        outs.append([_np(v) for v in (x, lf, z, lb)])
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            np.testing.assert_array_equal(a, b)


def _fast_case_chain(case, rng):
    """Default-shape relu chains that take the specialised kernel's FAST variant
    with 1, 2, 3 and 4 transformed dims per layer, NICE layers, conditioning and
    every hidden width the variant has (16, 32, 64)."""
    L = dfa.CouplingLayer
    if case == "af1_h64":      # d=4: n_af 1 (in 3), then 3 (in 1)
        return 4, 0, dfa.FlowChain(L(4, [2], hidden_dim=64, rng=rng), L(4, [1, 3, 4], hidden_dim=64, rng=rng))
    if case == "af4_h64":      # d=6: n_af 4 (in 2) twice
        return 6, 0, dfa.FlowChain(L(6, [1, 2, 3, 4], hidden_dim=64, rng=rng),
                                   L(6, [6, 2, 5, 3], hidden_dim=64, rng=rng))
    if case == "in4_h64":      # d=6: n_af 4 (in 2, folded), then 2 (in 4: no free k-slot) → FAST off
        return 6, 0, dfa.FlowChain(L(6, [1, 2, 3, 4], hidden_dim=64, rng=rng),
                                   L(6, [6, 2], hidden_dim=64, rng=rng))
    if case == "nice_h32":     # NICE + RNVP, conditioned (n=1), hidden 32
        return 5, 1, dfa.FlowChain(L(dfa.NICECouplingLayer, 5, [1, 2, 3], n=1, hidden_dim=32, rng=rng),
                                   L(5, [3, 4, 5], n=1, hidden_dim=32, rng=rng),
                                   L(dfa.NICECouplingLayer, 5, [5, 1, 2], n=1, hidden_dim=32, rng=rng))
    if case == "block_h16":    # CouplingBlocks, hidden 16
        return 5, 0, dfa.FlowChain.repeat(dfa.CouplingBlock, 2, 5, hidden_dim_s=16, hidden_dim_t=16, rng=rng)
    if case == "nice_h16":     # NICE + RNVP, conditioned, hidden 16: the small kernel's NICE layers
        return 5, 1, dfa.FlowChain(L(dfa.NICECouplingLayer, 5, [1, 2, 3], n=1, hidden_dim=16, rng=rng),
                                   L(5, [3, 4, 5], n=1, hidden_dim=16, rng=rng),
                                   L(dfa.NICECouplingLayer, 5, [5, 1, 2], n=1, hidden_dim=16, rng=rng))
    raise ValueError(case)


@pytest.mark.parametrize("case", ["af1_h64", "af4_h64", "in4_h64", "nice_h32", "block_h16", "nice_h16"])
def test_fast_variant_cases(cuda, case, monkeypatch, capfd):
    """FAST-variant tails for every output count: against the fp64 oracle, and
    bitwise against the non-FAST / unfolded plans of the same chain; the small-batch
    kernel (hidden 16 / 32) bitwise against the FAST kernel (DF_SMALL_MAX=0)."""
    import bench

    outs = []
    for env in ({"DF_DEBUG_LAUNCH": "1"}, {"DF_DEBUG_LAUNCH": "1", "DF_SMALL_MAX": "0"}, {"DF_NO_FAST": "1"},
                {"DF_NO_FOLD": "1"}, {"SPLIT": "1"}):
        for k in ("DF_NO_FAST", "DF_NO_FOLD", "DF_DEBUG_LAUNCH", "DF_F32_EXACT", "DF_SMALL_MAX"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            if k != "SPLIT":
                monkeypatch.setenv(k, v)
        if "SPLIT" not in env:   # bitwise comparisons among the exact-f32 kernels
            monkeypatch.setenv("DF_F32_EXACT", "1")
        rng = np.random.default_rng(11)
        d, n, chain = _fast_case_chain(case, rng)
        bench._init_nets(chain, rng)      # non-zero biases: the folded slot carries them
        rz = np.random.default_rng(12)
        B = 3000
        z = rz.standard_normal((d, B)).astype(np.float32)
        th = rz.random((n, B)).astype(np.float32) if n else None
        tth = _t(th, cuda) if n else None
        x, lf = dfa.forward(chain, _t(z, cuda), tth)
        zb, lb = dfa.backward(chain, x, tth)
        if "SPLIT" in env:   # the bf16x3 SPLIT kernel (hidden 32 / 64): f32-accurate, not bitwise
            assert _kernel_of(chain) in ((4,) if case in ("af1_h64", "af4_h64", "nice_h32") else
                                         (3,) if case in ("block_h16", "nice_h16") else (1, 2))
            xo, lo = O.forward(chain.to_spec(), z, th if n else np.zeros((0, B), np.float32), np.float64)
            assert close(_np(x), xo, RTOL)[0] and close(_np(lf), lo, RTOL)[0]
            assert np.all(np.abs(_np(lf) + _np(lb)) <= 2e-6 + 1e-5 * np.abs(_np(lf)))
            continue
        outs.append([_np(v) for v in (x, lf, zb, lb)])
        if "DF_DEBUG_LAUNCH" in env:
            import torch

            torch.cuda.synchronize()
            launches = capfd.readouterr().err
            # hidden-16 FAST chains of <= 4 layers at this batch run the small-batch kernel (df_small.hip),
            # whose outputs are bitwise the FAST kernel's (the comparisons below)
            small = case in ("block_h16", "nice_h16") and "DF_SMALL_MAX" not in env
            want = ("kernel uniform " if case == "in4_h64" else "kernel small " if small else
                    "kernel uniform-fast ")
            assert want in launches, launches
            xo, lo = O.forward(chain.to_spec(), z, th if n else np.zeros((0, B), np.float32), np.float64)
            assert close(_np(x), xo, RTOL)[0] and close(_np(lf), lo, RTOL)[0]
            # chain round trip: the inverse re-derives s from recomputed inputs, so the
            # cancellation is to rounding (runtests.jl:93 uses atol = 2f-6), not exact
            assert np.all(np.abs(_np(lf) + _np(lb)) <= 2e-6 + 1e-5 * np.abs(_np(lf)))
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("B", [0, 1, 7, 127, 128, 129, 1000, 4095])
def test_ragged_batches(cuda, B):
    spec, g, _ = G.load("cfg1")
    chain = spec_to_element(spec)
    z = g["z"][:, :B]
    th = g["theta"][:, :B]
    x, l = dfa.forward(chain, _t(z, cuda), _t(th, cuda))
    assert tuple(x.shape) == (5, B) and tuple(l.shape) == (B,)
    if B:
        assert close(_np(x), g["x_fwd"][:, :B], RTOL)[0]
        assert close(_np(l), g["ldj_fwd"][:B], RTOL)[0]


def test_nd_dims_and_numpy_io(cuda):
    """(d, dims...) arrays: ldj has shape dims (RNVP.jl:180 dropdims)."""
    spec, g, _ = G.load("cfg2")
    chain = spec_to_element(spec)
    z = g["z"][:, :70].reshape(5, 2, 5, 7, order="F")
    x, l = dfa.forward(chain, z)          # numpy in → numpy out
    assert x.shape == (5, 2, 5, 7) and l.shape == (2, 5, 7)
    assert close(x.reshape(5, 70, order="F"), g["x_fwd"][:, :70], RTOL)[0]
    assert close(l.reshape(70, order="F"), g["ldj_fwd"][:70], RTOL)[0]


@pytest.mark.parametrize("act", ["tanh", "sigmoid", "softplus", "logcosh", "leakyrelu", "elu", "swish", "identity"])
def test_activations(cuda, act):
    rng = np.random.default_rng(7)
    ch = dfa.FlowChain(dfa.CouplingLayer(5, [2, 4], hidden_dim=32, σ=act, rng=rng),
                       dfa.CouplingLayer(5, [1, 3, 5], hidden_dim=32, σ=act, rng=rng))
    z = rng.standard_normal((5, 300)).astype(np.float32)
    x, l = dfa.forward(ch, _t(z, cuda))
    xo, lo = O.forward(ch.to_spec(), z, np.zeros((0, 300)), np.float64)
    assert close(_np(x), xo, RTOL)[0] and close(_np(l), lo, RTOL)[0]


def test_nice_and_custom_nets(cuda):
    """NICE layers and hand-built conditioners of mixed widths (docs/src/documentation.md:99-105)."""
    rng = np.random.default_rng(8)
    d, n = 7, 1
    s_net = dfa.Chain([dfa.Dense.init(5, 32, "sigmoid", rng=rng), dfa.Dense.init(32, 16, "relu", rng=rng),
                       dfa.Dense.init(16, 3, rng=rng)])
    t_net = dfa.Chain([dfa.Dense.init(5, 12, "relu", rng=rng), dfa.Dense.init(12, 16, "logcosh", rng=rng),
                       dfa.Dense.init(16, 32, "relu", rng=rng), dfa.Dense.init(32, 3, rng=rng)])
    ax = dfa.CouplingAxes.from_mask(d, [6, 2, 4], n=n)
    rn = dfa.CouplingLayer(s_net, t_net, ax)
    nice = dfa.CouplingLayer(dfa.NICECouplingLayer, d, 3, n=n, rng=rng)
    ch = dfa.FlowChain(rn, nice, dfa.CouplingBlock.build(d, 4, n=n, rng=rng, hidden_dim=48))
    z = rng.standard_normal((d, 513)).astype(np.float32)
    th = rng.random((n, 513)).astype(np.float32)
    x, l = dfa.forward(ch, _t(z, cuda), _t(th, cuda))
    xo, lo = O.forward(ch.to_spec(), z, th, np.float64)
    assert close(_np(x), xo, RTOL)[0] and close(_np(l), lo, RTOL)[0]
    zb, lb = dfa.backward(ch, x, _t(th, cuda))
    assert close(_np(zb), z, RTOL)[0]
    assert np.all(np.abs(_np(l) + _np(lb)) <= 1e-5 * np.maximum(1, np.abs(_np(l))))


def test_wide_af_mfma_output_path(cuda):
    """More than 4 transformed dims → the MFMA output path (n_af up to 32)."""
    rng = np.random.default_rng(9)
    ch = dfa.FlowChain.repeat(dfa.CouplingBlock, 2, 40, 20, n=3, hidden_dim_s=64, hidden_dim_t=64, rng=rng)
    z = rng.standard_normal((40, 777)).astype(np.float32)
    th = rng.random((3, 777)).astype(np.float32)
    x, l = dfa.forward(ch, _t(z, cuda), _t(th, cuda))
    xo, lo = O.forward(ch.to_spec(), z, th, np.float64)
    assert close(_np(x), xo, RTOL)[0] and close(_np(l), lo, RTOL)[0]


def test_full_size_roundtrip_properties(cuda):
    """BASELINE config 2 at its full size (B = 2^20): size-independent
    properties — inverse(forward(z)) ≈ z, ldj_f + ldj_b ≈ 0, finite, and a
    sampled subset against the oracle."""
    import torch

    spec, _, _ = G.load("cfg2")
    chain = spec_to_element(spec)
    B = 1 << 20
    gen = torch.Generator(device=cuda).manual_seed(1)
    z = torch.randn(B, 5, device=cuda, generator=gen).T
    x, lf = dfa.forward(chain, z)
    zb, lb = dfa.backward(chain, x)
    assert torch.isfinite(x).all() and torch.isfinite(lf).all()
    err = (zb - z).abs().max().item()
    assert err <= 1e-4, err
    assert (lf + lb).abs().max().item() <= 1e-5
    idx = torch.randint(0, B, (2048,), device=cuda, generator=gen)
    zs = _np(z[:, idx])
    xo, lo = O.forward(spec, zs, np.zeros((0, zs.shape[1])), np.float64)
    assert close(_np(x[:, idx]), xo, RTOL)[0] and close(_np(lf[idx]), lo, RTOL)[0]


def test_deterministic_repeat(cuda):
    spec, g, _ = G.load("cfg2")
    chain = spec_to_element(spec)
    a, la = dfa.forward(chain, _t(g["z"], cuda))
    b, lb = dfa.forward(chain, _t(g["z"], cuda))
    np.testing.assert_array_equal(_np(a), _np(b))
    np.testing.assert_array_equal(_np(la), _np(lb))


def test_sample_shape_and_theta_tuple(cuda):
    """test/runtests.jl:118-120: size(sample(flow, (2,5,7), (-1f0,))) == (5,2,5,7)."""
    spec, g, meta = G.load("cfg1")
    md = dfa.MetaData("", 5, 1, g["theta_min"], g["theta_max"])
    flow = dfa.Flow(spec_to_element(spec), metadata=md)
    s = dfa.sample(flow, (2, 5, 7), (-1.0,))
    assert tuple(s.shape) == (5, 2, 5, 7)
    import torch

    assert torch.isfinite(s).all()


def test_errors_are_loud(cuda):
    spec, g, _ = G.load("cfg1")
    chain = spec_to_element(spec)
    with pytest.raises(AssertionError):
        dfa.forward(chain, _t(g["z"][:4], cuda), _t(g["theta"], cuda))   # wrong d
    with pytest.raises(AssertionError):
        dfa.forward(chain, _t(g["z"], cuda), None)                        # missing θ


# ---------------------------------------------------------------------------
# forward! and sample: value parity (src/affine/RNVP.jl:190-205,
# src/Chains.jl:187-197, src/norm/Normalization.jl:95-103, src/Flows.jl:157-192)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_chain_forward_inplace_against_oracle(cuda, name):
    """df_chain_forward_inplace (θ used as given) against O.forward_inplace, and
    bitwise the x of df_chain_forward."""
    spec, g, meta = G.load(name)
    chain = spec_to_element(spec)
    th = _t(g["theta"], cuda) if meta["n"] > 0 else None
    zz = _t(g["z"], cuda)
    dfa.forward_(chain, zz, th)
    zo = np.array(g["z"], np.float64)
    O.forward_inplace(spec, zo, g["theta"] if meta["n"] > 0 else np.zeros((0, meta["B"])), np.float64)
    ok, r = close(_np(zz), zo, RTOL)
    assert ok, r
    x, _ = dfa.forward(chain, _t(g["z"], cuda), th)
    np.testing.assert_array_equal(_np(zz), _np(x))


def test_flow_forward_inplace_theta_tuple_and_normalization(cuda):
    """df_flow_forward_inplace on the README chain (NormalizationLayer last):
    raw θ normalised in-kernel, NTuple θ broadcast to every point."""
    spec, g, meta = G.load("cfg1")
    flow = dfa.Flow(spec_to_element(spec), metadata=dfa.MetaData("", 5, 1, g["theta_min"], g["theta_max"]))
    B = meta["B"]
    zz = _t(g["z"], cuda)
    flow.forward_(zz, _t(g["theta_raw"], cuda))
    zo = np.array(g["z"], np.float64)
    O.forward_inplace(spec, zo, O.normalize_input(g["theta_raw"], g["theta_min"], g["theta_max"]), np.float64)
    ok, r = close(_np(zz), zo, RTOL)
    assert ok, r
    # NTuple θ = (2f0,): collect(θ) .* ones(T, (1, dims...))  (src/Flows.jl:182)
    zz = _t(g["z"], cuda)
    flow.forward_(zz, (2.0,))
    zo = np.array(g["z"], np.float64)
    th = O.normalize_input(np.full((1, B), 2.0, np.float32), g["theta_min"], g["theta_max"])
    O.forward_inplace(spec, zo, th, np.float64)
    ok, r = close(_np(zz), zo, RTOL)
    assert ok, r


@pytest.mark.parametrize("theta", ["array", "tuple"])
def test_sample_values_against_oracle(cuda, theta):
    """sample(flow, dims, θ) through df_flow_sample (device Philox draw + fused
    forward!): the same draw read back with df_random_normal (same seed) through
    O.forward_inplace (src/Flows.jl:174-185; Julia's Xoshiro stream itself cannot be
    matched), and bitwise the library's own forward! of that draw."""
    import torch

    spec, g, meta = G.load("cfg1")
    flow = dfa.Flow(spec_to_element(spec), metadata=dfa.MetaData("", 5, 1, g["theta_min"], g["theta_max"]))
    dims = (3, 200)
    B = 600
    if theta == "tuple":
        th_arg, th_raw = (-1.0,), np.full((1, B), -1.0, np.float32)
    else:
        th_raw = np.random.default_rng(3).uniform(-1, 2, (1, B)).astype(np.float32)
        th_arg = th_raw.reshape((1,) + dims, order="F")     # logical (n, dims...), Julia memory order
    s = dfa.sample(flow, dims, th_arg, seed=77)
    buf = torch.empty(5 * B, dtype=torch.float32, device=cuda)
    flow.hip().random_normal(buf, 5 * B, 77)
    rn = _np(buf).reshape(5, B, order="F").astype(np.float64)
    r2 = buf.reshape(B, 5).T                                 # logical (5, B) view, Julia order
    flow.forward_(r2, _t(th_raw, cuda))
    O.forward_inplace(spec, rn, O.normalize_input(th_raw, g["theta_min"], g["theta_max"]), np.float64)
    assert tuple(s.shape) == (5,) + dims
    sv = _np(s).reshape(5, B, order="F")
    ok, rr = close(sv, rn, RTOL)
    assert ok, rr
    np.testing.assert_array_equal(sv, _np(r2))


def test_device_normal_draw_moments(cuda):
    """df_random_normal (the base draw of df_flow_sample, MvNormal(0, I) of
    src/Flows.jl:114): moments of 2^22 draws, determinism in (seed, offset), and a
    different stream for another seed or offset."""
    import torch

    spec, g, meta = G.load("cfg1")
    h = spec_to_element(spec).hip()
    N = 1 << 22
    a = torch.empty(N, dtype=torch.float32, device=cuda)
    b = torch.empty(N, dtype=torch.float32, device=cuda)
    h.random_normal(a, N, 12345)
    z = _np(a).astype(np.float64)
    assert np.all(np.isfinite(z))
    assert abs(z.mean()) < 3e-3 and abs(z.var() - 1.0) < 3e-3
    assert abs(np.mean(z ** 4) - 3.0) < 3e-2                     # kurtosis of N(0, 1)
    assert abs(np.mean(np.abs(z) < 1.0) - 0.682689) < 2e-3
    assert abs(np.mean(np.abs(z) < 2.0) - 0.954500) < 1e-3
    h.random_normal(b, N, 12345)
    np.testing.assert_array_equal(_np(a), _np(b))
    h.random_normal(b, N, 12346)
    assert np.mean(_np(a) == _np(b)) < 1e-3
    h.random_normal(b, N - 4, 12345, offset=1)                   # counter offset: the stream shifted by 4
    np.testing.assert_array_equal(_np(a)[4:], _np(b)[:N - 4])
    # ragged counts: the draw of a prefix is the prefix of the draw
    h.random_normal(b, 1001, 12345)
    np.testing.assert_array_equal(_np(a)[:1001], _np(b)[:1001])


def test_theta_row_with_max_equal_min(cuda):
    """normalize_input sets rows with θ_max == θ_min to 0 (src/Data.jl:216):
    forward, backward, forward! and logpdf of a 2-condition flow whose second
    condition is constant."""
    rng = np.random.default_rng(21)
    ch = dfa.FlowChain(dfa.CouplingLayer(5, [1, 2, 3], n=2, hidden_dim=32, rng=rng),
                       dfa.CouplingLayer(5, [4, 5], n=2, hidden_dim=32, σ="tanh", rng=rng))
    import bench

    bench._init_nets(ch, rng)
    B = 1500
    z = rng.standard_normal((5, B)).astype(np.float32)
    th_raw = np.vstack([rng.uniform(-1, 2, B), np.full(B, 3.0)]).astype(np.float32)
    tmin, tmax = np.array([-1.0, 3.0], np.float32), np.array([2.0, 3.0], np.float32)
    flow = dfa.Flow(ch, metadata=dfa.MetaData("", 5, 2, tmin, tmax))
    thn = O.normalize_input(th_raw, tmin, tmax)
    assert np.all(thn[1] == 0)
    spec = ch.to_spec()
    x, lf = flow.forward(_t(z, cuda), _t(th_raw, cuda))
    xo, lo = O.forward(spec, z, thn, np.float64)
    assert close(_np(x), xo, RTOL)[0] and close(_np(lf), lo, RTOL)[0]
    zb, lb = flow.backward(_t(xo.astype(np.float32), cuda), _t(th_raw, cuda))
    zo, lbo = O.backward(spec, xo.astype(np.float32), thn, np.float64)
    assert close(_np(zb), zo, RTOL)[0] and close(_np(lb), lbo, RTOL)[0]
    zz = _t(z, cuda)
    flow.forward_(zz, _t(th_raw, cuda))
    assert close(_np(zz), xo, RTOL)[0]
    lp = dfa.logpdf(flow, _t(xo.astype(np.float32), cuda), _t(th_raw, cuda))
    lpo = O.flow_logpdf(spec, xo.astype(np.float32), thn, np.float64)
    assert close(_np(lp), lpo, RTOL)[0]


# ---------------------------------------------------------------------------
# strict element-wise relative error (no max-scaled floor)
# ---------------------------------------------------------------------------

STRICT_FLOOR = 1e-3     # judged where |expected| > 1e-3
STRICT_RTOL = 1e-5


def strict_rel(a, b, floor=STRICT_FLOOR):
    """Per-element |a-b|/|b| where |b| > floor: (max, p99.9, p99, fraction > 1e-5, n)."""
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    m = np.abs(b) > floor
    if not m.any():
        return 0.0, 0.0, 0.0, 0.0, 0
    r = np.abs(a[m] - b[m]) / np.abs(b[m])
    return (float(r.max()), float(np.percentile(r, 99.9)), float(np.percentile(r, 99)),
            float((r > STRICT_RTOL).mean()), int(m.sum()))


def _kernel_of(chain):
    return chain.hip().info.kernel


@pytest.mark.parametrize("name", ["cfg2", "fast_h32", "cfg4"])
def test_split_variant_accuracy(cuda, name, monkeypatch):
    """The SPLIT variant (df_uniform_impl.h: first and hidden Dense on bf16 MFMA
    with both operands in three bf16 planes, six products, f32 accumulation) is an
    f32-accurate evaluation: against the fp64 truth its strict per-element error
    is within 1.5× that of the exact-f32 MFMA kernel (DF_F32_EXACT=1) at the
    median and the 99th percentile, for x and ldj in both directions; the worst
    (ill-conditioned) element within 2× the worst of the exact-f32 kernel and of
    Flux's op order in fp32, and — against the exact-f32 kernel alone — the
    99.9th percentile within 2× and the worst element within 3× or under 1e-5."""
    th = None
    if name in ("cfg2", "cfg4"):
        spec, g, meta = G.load(name)
        z, xin = g["z"], g["x_in"]
        xo, lo = g["x_fwd"], g["ldj_fwd"]
        zo, lbo = g["z_bwd"], g["ldj_bwd"]
        th = g["theta"] if meta["n"] > 0 else None
    else:  # hidden 32 (HT = 2), 4 RNVP layers on d = 6
        rng = np.random.default_rng(7)
        ch = dfa.FlowChain.repeat(dfa.CouplingBlock, 2, 6, hidden_dim_s=32, hidden_dim_t=32, rng=rng)
        spec = ch.to_spec()
        z = rng.standard_normal((6, 3000))
        xo, lo = O.forward(spec, z, np.zeros((0, 3000)), np.float64)
        xin = xo.astype(np.float32)
        zo, lbo = O.backward(spec, xin.astype(np.float64), np.zeros((0, 3000)), np.float64)
        z = z.astype(np.float32)
    th_np = th if th is not None else np.zeros((0, z.shape[1]), np.float32)
    ref32 = list(O.forward(spec, z, th_np, np.float32)) + list(O.backward(spec, xin, th_np, np.float32))
    wide = name == "cfg4"
    res = {}
    for exact in ("0", "1"):
        monkeypatch.setenv("DF_F32_EXACT", exact)
        chain = spec_to_element(spec)
        assert _kernel_of(chain) == ((5 if wide else 3) if exact == "1" else (6 if wide else 4))
        tth = _t(th, cuda) if th is not None else None
        x, lf = dfa.forward(chain, _t(z, cuda), tth)
        zb, lb = dfa.backward(chain, _t(xin, cuda), tth)
        res[exact] = [_np(v) for v in (x, lf, zb, lb)]
    print(f"strict relative error vs fp64 ({name}): quantity split(median, p99, p99.9, max) | exact-f32(same)")
    for i, (key, truth) in enumerate((("x", xo), ("ldj", lo), ("z", zo), ("ldj_bwd", lbo))):
        es = strict_rel(res["0"][i], truth)
        ee = strict_rel(res["1"][i], truth)
        a = np.abs(np.asarray(truth, np.float64))
        m = a > 1e-3
        med_s = float(np.median(np.abs(res["0"][i].astype(np.float64) - truth)[m] / a[m]))
        med_e = float(np.median(np.abs(res["1"][i].astype(np.float64) - truth)[m] / a[m]))
        print(f"  {key}: ({med_s:.3g}, {es[2]:.3g}, {es[1]:.3g}, {es[0]:.3g}) | "
              f"({med_e:.3g}, {ee[2]:.3g}, {ee[1]:.3g}, {ee[0]:.3g})")
        # the worst element is an ill-conditioned sample whose error depends on the
        # summation order: judged, as in test_strict_elementwise_relative_error, against
        # 2× the worst of the exact-f32 kernel and of Flux's own op order in fp32
        ef = strict_rel(ref32[i], truth)
        assert med_s <= 1.5 * med_e + 1e-8, (key, med_s, med_e)
        assert es[2] <= 1.5 * ee[2] + 1e-8, (key, es, ee)
        assert es[0] <= max(1e-5, 2.0 * max(ee[0], ef[0])), (key, es, ee, ef)
        # SPLIT-specific tail bounds, against the exact-f32 kernel alone (a regression of
        # the split cannot hide under the worst element of Flux's fp32 op order): the
        # 99.9th percentile within 2x, the worst element within 3x or under 1e-5
        # (round 2: worst ratios 2.2x on fast_h32 ldj_bwd, 6.2x on cfg2 ldj at 4.3e-6)
        assert es[1] <= 2.0 * ee[1] + 1e-8, (key, es, ee)
        assert es[0] <= max(1e-5, 3.0 * ee[0]), (key, es, ee)


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_strict_elementwise_relative_error(cuda, name):
    """north_star: 1e-5 relative fp32, judged per element (no max-scaled floor)
    wherever |expected| > 1e-3, for x, ldj (both directions) and logpdf on every
    golden fixture, against the fp64 truth.

    Measured (GPU, round 2): the fp32 evaluation of the reference's own op
    sequence (the oracle's Flux-like fp32 mode: sgemm, broadcast bias/σ, exp)
    is itself NOT within 1e-5 of the exact value on every element: x = z·e^s + t
    cancels where the two terms nearly cancel (cfg1 x: worst 1.7e-4 for Flux-in-
    fp32), and ldj = Σ s over 16 layers of hidden-256 nets carries the fp32
    rounding of every s (cfg4 ldj: worst 2.4e-4).  The worst element is one
    ill-conditioned sample, and which one depends on the summation order (MFMA
    k-order chains here, blocked sgemm in Flux).  So, per quantity:
      * the 99th percentile of the strict error is ≤ 1e-5 (north_star's bar for
        all but the ill-conditioned 1 %);
      * the worst element is ≤ max(1e-5, 2 × Flux-in-fp32's worst);
      * the fraction of elements over 1e-5 is ≤ max(1e-3, 2 × Flux-in-fp32's)."""
    spec, g, meta = G.load(name)
    chain = spec_to_element(spec)
    n = meta["n"]
    th_np = g["theta"] if n > 0 else np.zeros((0, meta["B"]), np.float32)
    th = _t(g["theta"], cuda) if n > 0 else None
    x, lf = dfa.forward(chain, _t(g["z"], cuda), th)
    z, lb = dfa.backward(chain, _t(g["x_in"], cuda), th)
    flow = dfa.Flow(spec_to_element(spec), metadata=dfa.MetaData("", meta["d"], n, g["theta_min"], g["theta_max"]))
    lp = dfa.logpdf(flow, _t(g["x_in"], cuda), _t(g["theta_raw"], cuda) if n > 0 else None)
    x32, l32 = O.forward(spec, g["z"], th_np, np.float32)
    z32, lb32 = O.backward(spec, g["x_in"], th_np, np.float32)
    lp32 = O.flow_logpdf(spec, g["x_in"], th_np, np.float32)
    bad = {}
    print(f"strict relative error {name} vs fp64 truth: quantity gpu(max, p99.9, p99, frac>1e-5) | "
          "Flux-like fp32(same) | n")
    for key, got, ref32 in (("x_fwd", x, x32), ("ldj_fwd", lf, l32), ("z_bwd", z, z32), ("ldj_bwd", lb, lb32),
                            ("logpdf", lp, lp32)):
        eg = strict_rel(_np(got), g[key])
        er = strict_rel(ref32, g[key])
        print(f"  {key}: ({eg[0]:.3g}, {eg[1]:.3g}, {eg[2]:.3g}, {eg[3]:.2g}) | "
              f"({er[0]:.3g}, {er[1]:.3g}, {er[2]:.3g}, {er[3]:.2g}) | {eg[4]}")
        if (eg[2] > STRICT_RTOL or eg[0] > max(STRICT_RTOL, 2.0 * er[0])
                or eg[3] > max(1e-3, 2.0 * er[3])):
            bad[key] = (eg, er)
    assert not bad, bad


def test_chain_set_weights(cuda):
    """df_chain_set_weights: an inference handle takes new parameters of the same
    structure (weights, biases, NormalizationLayer bounds); a different
    structure is refused."""
    import bench

    spec, g, meta = G.load("cfg1")
    chain = spec_to_element(spec)
    hc = chain.hip()
    rng = np.random.default_rng(31)
    other = bench.build_chain("cfg1", seed=31)
    hc.set_weights(other.layers)
    th = _t(g["theta"], cuda)
    x, l = hc.apply("forward", _t(g["z"], cuda), th)
    xo, lo = O.forward(other.to_spec(), g["z"], g["theta"], np.float64)
    assert close(_np(x), xo, RTOL)[0] and close(_np(l), lo, RTOL)[0]
    wrong = dfa.FlowChain(dfa.CouplingLayer(5, [1, 2, 3], n=1, hidden_dim=32, rng=rng))
    with pytest.raises((AssertionError, dfa.ArgumentError)):
        hc.set_weights(wrong.layers)


@pytest.mark.parametrize("B", [1, 31, 32, 33, 4096, 5000])
def test_small_kernel_bitwise_fast_kernel(cuda, B, monkeypatch, capfd):
    """The small-batch kernel (df_small.hip: state rows in registers, weights loaded
    from the blob, no LDS) against the FAST kernel it replaces at small batches
    (DF_SMALL_MAX=0): forward, forward!, inverse, per-sample logpdf and the inverse
    pass's per-layer outputs (training snapshots, via a gradient) bitwise; the
    fp64 Σ logpdf to rounding of its summation order.  Both forms of the small kernel:
    the s- and t-nets of a layer on two waves (default) and on one (DF_SMALL_WAVES=1)."""
    import torch

    from densityflows_amd.train import Adam, HIPTrainer

    spec, g, meta = G.load("cfg1")
    z = np.ascontiguousarray(g["z"][:, :B]) if B <= g["z"].shape[1] else \
        np.random.default_rng(B).standard_normal((5, B)).astype(np.float32)
    th = np.random.default_rng(B + 1).uniform(-1, 2, (1, B)).astype(np.float32)
    res = {}
    for mode in ("small", "small1", "fast"):
        monkeypatch.delenv("DF_SMALL_MAX", raising=False)
        monkeypatch.delenv("DF_SMALL_WAVES", raising=False)
        if mode == "fast":
            monkeypatch.setenv("DF_SMALL_MAX", "0")
        if mode == "small1":
            monkeypatch.setenv("DF_SMALL_WAVES", "1")
        monkeypatch.setenv("DF_DEBUG_LAUNCH", "1")
        chain = spec_to_element(spec)
        flow = dfa.Flow(chain, metadata=dfa.MetaData("", 5, 1, g["theta_min"], g["theta_max"]))
        x, lf = dfa.forward(chain, _t(z, cuda), _t(th, cuda))
        zb, lb = dfa.backward(chain, x, _t(th, cuda))
        zz = _t(z, cuda).clone()
        flow.forward_(zz, _t(th, cuda))
        lp = dfa.logpdf(flow, x, _t(th, cuda))
        s, _ = flow.hip().logpdf_sum(x, _t(th, cuda))
        tr = HIPTrainer(chain.hip(), Adam())
        lps = torch.zeros(1, dtype=torch.float64, device=cuda)
        xflat = x.T.contiguous().reshape(-1)
        tr.gradient(xflat, _t(th, cuda).T.contiguous().reshape(-1), B, B, lps)
        torch.cuda.synchronize()
        launches = capfd.readouterr().err
        assert ("kernel small " in launches) == (mode != "fast"), launches
        res[mode] = ([_np(v) for v in (x, lf, zb, lb, zz, lp)], float(s.item()), tr.grad().cpu().numpy().copy(),
                     float(lps.item()))
        monkeypatch.delenv("DF_DEBUG_LAUNCH", raising=False)
    for m in ("small", "small1"):
        for a, b in zip(res[m][0], res["fast"][0]):
            np.testing.assert_array_equal(a, b)
        np.testing.assert_allclose(res[m][1], res["fast"][1], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(res[m][3], res["fast"][3], rtol=1e-12, atol=1e-9)
        # the gradient reads the inverse pass's snapshots: equal snapshots → equal gradient
        np.testing.assert_array_equal(res[m][2], res["fast"][2])
