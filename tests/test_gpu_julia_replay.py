"""The Julia front-end's train! / sample call sequence, replayed through ctypes on the GPU.

tests/julia_replay.py re-enacts densityflows.jl_amd/julia/DensityFlowsHIP.jl ccall for
ccall (tests/test_julia_shim.py checks the symbol order statically).  Here it runs the
reference's conditional README chain (test/runtests.jl:97-121: θ ∈ {−1, 2}, the
datatest.jld2 fixture) through

    sample(flow, dims, θ)  →  train!(flow, data, Adam(1f-3); batchsize=64, shuffle=false)
                           →  sample(flow, dims, θ)

i.e. the θ bounds are on the chain (set by the first sample) while train! runs — the
case where a step that normalised θ itself would normalise normalized_training_data
twice.  Expected values: the oracle's epoch loop (nll_and_grad + Adam on the same
normalised mini-batches, then the full train / valid losses; the criterion of
test_gpu_train.test_train_epochs_match_oracle_loop), the oracle forward! of the same
device draw for both samples, and bitwise the Python mirror's train_ (same kernels,
same θ) for the parameters.
"""
import numpy as np
import pytest

import densityflows_amd as dfa
import julia_replay as J
from densityflows_amd.train import Adam, load_trainables, setup, train_, trainables
from helpers import close
from oracle import flow_oracle as O
from test_gpu_train import _datatest_flow, _flat_oracle_grads

pytestmark = pytest.mark.gpu

EPOCHS = 2
BS = 64


def _draw(seed, count):
    """The base draw of df_flow_sample (df_random_normal, same seed / offset 0), on the host."""
    import ctypes as C

    p = J._dev(4 * count)
    J.check(J.lib().df_random_normal(p, C.c_int64(count), C.c_uint64(seed), C.c_uint64(0), J.NULL),
            "df_random_normal")
    r = np.empty(count, np.float32)
    J._d2h(r, p)
    J._free(p)
    return r


def _oracle_epochs(seed):
    """The oracle's train! on the same normalised, contiguous mini-batches."""
    data, chain_o, flow_o = _datatest_flow(seed=seed)
    md = flow_o.metadata
    x_tr, th_tr = data.training_data()
    x_va, th_va = data.validation_data()
    thn_tr = O.normalize_input(th_tr, md.theta_min, md.theta_max)
    thn_va = O.normalize_input(th_va, md.theta_min, md.theta_max)
    p = trainables(chain_o).astype(np.float32)
    st = [np.zeros_like(p), np.zeros_like(p), (np.float32(0.9), np.float32(0.999))]
    spec = chain_o.to_spec()
    tl, vl = [], []
    N = x_tr.shape[1]
    for _ in range(EPOCHS):
        for b0 in range(0, N, BS):
            _, g = O.nll_and_grad(spec, x_tr[:, b0:b0 + BS], thn_tr[:, b0:b0 + BS])
            O.adam_update(p, _flat_oracle_grads(spec, g).astype(np.float32), st)
            load_trainables(chain_o, p)
            spec = chain_o.to_spec()
        tl.append(-float(np.mean(O.flow_logpdf(spec, x_tr, thn_tr, np.float64))))
        vl.append(-float(np.mean(O.flow_logpdf(spec, x_va, thn_va, np.float64))))
    return p, spec, tl, vl


def test_julia_sample_train_sample_sequence(cuda):
    J.CALLS.clear()
    J.__init__()
    data, chain, flow_py = _datatest_flow(seed=3)
    spec0 = chain.to_spec()
    md = flow_py.metadata
    c = J.HIPFlowChain(chain)
    flow = J.Flow(c, md)
    dims = (4, 75)
    B = int(np.prod(dims))
    th_raw = np.where(np.arange(B) % 2 == 0, -1.0, 2.0).astype(np.float32).reshape((1,) + dims, order="F")
    thn = O.normalize_input(th_raw.reshape(1, B, order="F"), md.theta_min, md.theta_max)
    try:
        # 1. sample (sets the chain's θ bounds)
        s0 = J._hip_sample(11, flow, dims, th_raw, False)
        z = _draw(11, 5 * B).reshape(5, B, order="F").astype(np.float64)
        ref0 = z.copy()
        O.forward_inplace(spec0, ref0, thn, np.float64)
        ok, r = close(s0.reshape(5, B, order="F"), ref0)
        assert ok, ("sample before train!", r)
        assert c.bounds is not None

        # 2. train!(flow, data, Adam(1f-3)) with the bounds set
        n0 = len(J.CALLS)
        assert J.train_bang(flow, data, Adam(1e-3), epochs=EPOCHS, batchsize=BS, shuffle=False,
                            verbose=False) is None
        train_calls = J.CALLS[n0:]
        n_batches = -(-data.training_data()[0].shape[1] // BS)
        assert train_calls.count("df_train_step") == EPOCHS * n_batches
        assert train_calls.count("df_chain_logpdf_sum") == 2 * EPOCHS
        assert not any(s.startswith("df_flow_") for s in train_calls), set(train_calls)

        p_ref, spec_ref, tl, vl = _oracle_epochs(seed=3)
        print("train_loss", flow.train_loss, tl, "valid_loss", flow.valid_loss, vl)
        np.testing.assert_allclose(flow.train_loss, tl, rtol=2e-4)
        np.testing.assert_allclose(flow.valid_loss, vl, rtol=2e-4)
        dp = np.abs(c.params - p_ref)
        print("param |Δ| median / p99 / max", np.median(dp), np.quantile(dp, 0.99), dp.max())
        # measured on the GPU: median 0, p99 3.0e-8, max 6.0e-8 (gpurun_out/r05a)
        assert np.quantile(dp, 0.99) <= 2e-6 and dp.max() <= 1e-5

        # the Python mirror's train_ (θ raw, normalised in the kernels with the bounds) on
        # the same data gives bitwise the same parameters and losses
        data2, chain2, flow2 = _datatest_flow(seed=3)
        train_(flow2, data2, setup(Adam(1e-3), flow2), epochs=EPOCHS, batchsize=BS, shuffle=False,
               verbose=False, graphs=False)
        np.testing.assert_array_equal(c.params, trainables(chain2))
        np.testing.assert_array_equal(np.float32(flow.train_loss), np.float32(flow2.train_loss))

        # 3. sample again: the trained parameters, the same draw
        s1 = J._hip_sample(11, flow, dims, th_raw, False)
        ref1 = z.copy()
        O.forward_inplace(spec_ref, ref1, thn, np.float64)
        ok, r = close(s1.reshape(5, B, order="F"), ref1, 1e-4)
        assert ok, ("sample after train!", r)
        assert not np.array_equal(s0, s1)

        # 3b. weight export (src/Loading.jl:78-96,324-346): the device vector
        # written into a FRESH mirror model by copy_trainables! (Flux.trainables order), a
        # chain re-created from that model, and its forward bitwise the trained chain's
        _, chain_new, _ = _datatest_flow(seed=99)            # same structure, other weights
        assert not np.array_equal(trainables(chain_new), c.params)
        J.copy_trainables_bang(chain_new, c.params)
        np.testing.assert_array_equal(trainables(chain_new), c.params)
        for D_new, D_py in zip(chain_new.layers[0].s_net, chain2.layers[0].s_net):  # per Dense, mirror walk
            np.testing.assert_array_equal(D_new.W, D_py.W)
        c_new = J.HIPFlowChain(chain_new)
        try:
            x_tr, th_tr = data.training_data()
            thn_tr = J.normalize_input(th_tr, md.theta_min, md.theta_max)
            xa, la = J.forward(c, x_tr, thn_tr)
            xb_, lb_ = J.forward(c_new, x_tr, thn_tr)
            np.testing.assert_array_equal(xa, xb_)
            np.testing.assert_array_equal(la, lb_)
            za, lza = J.backward(c, x_tr, thn_tr)
            zb2, lzb = J.backward(c_new, x_tr, thn_tr)
            np.testing.assert_array_equal(za, zb2)
            np.testing.assert_array_equal(lza, lzb)
        finally:
            c_new.finalize()
        with pytest.raises(IndexError):                      # copyto! past the end (BoundsError)
            J.copy_trainables_bang(chain_new, c.params[:-1])
        with pytest.raises(AssertionError):                  # DimensionMismatch: a longer vector
            J.copy_trainables_bang(chain_new, np.concatenate([c.params, np.zeros(1, np.float32)]))

        # 4. the model-level calls the shim exposes, θ as given, bounds still set
        x_va, th_va = data.validation_data()
        thn_va = J.normalize_input(th_va, md.theta_min, md.theta_max)
        zb, ldj = J.backward(c, x_va, thn_va)
        zo, lo = O.backward(spec_ref, x_va, thn_va, np.float64)
        assert close(zb, zo, 1e-4)[0] and close(ldj, lo, 1e-4)[0]
        nll = J.flow_nll(c, None, x_va, thn_va)
        np.testing.assert_allclose(nll, flow.valid_loss[-1], rtol=1e-6)
        # a second train! epoch from the HIPTrainer kept on the chain (same Adam key)
        t_before = c.trainer
        J.train_bang(flow, data, Adam(1e-3), epochs=1, batchsize=BS, shuffle=False, verbose=False)
        assert c.trainer is t_before and len(flow.train_loss) == EPOCHS + 1
    finally:
        c.finalize()


def test_trainer_theta_input_modes(cuda):
    """df_train_set_theta_input: GIVEN never reads the chain's bounds, RAW requires
    them, AUTO follows them (ABI 3 behaviour); a captured graph step is re-captured
    when the effective convention changes (bounds set after capture)."""
    import ctypes as C

    import torch

    from densityflows_amd import _lib
    from densityflows_amd.train import HIPTrainer
    from test_gpu_train import _dev, _inputs, _setup

    spec, chain, d, n = _setup("readme")
    x, th = _inputs(d, n, 512, seed=9)
    tmin, tmax = np.array([-1.0], np.float32), np.array([2.0], np.float32)
    thn = O.normalize_input(th, tmin, tmax)

    def grad(tr, theta):
        lp = torch.zeros(1, dtype=torch.float64, device=cuda)
        tr.gradient(_dev(x, cuda), _dev(theta, cuda), 512, 512, lp)
        torch.cuda.synchronize()
        return tr.grad().cpu().numpy().copy()

    h = chain.hip()
    tr = HIPTrainer(h, Adam())
    g_given = grad(tr, thn)                               # no bounds: θ as given
    h.set_theta_bounds(tmin, tmax)
    g_auto_raw = grad(tr, th)                             # AUTO + bounds: raw θ normalised
    np.testing.assert_array_equal(g_given, g_auto_raw)
    _lib.check(tr.lib.df_train_set_theta_input(tr.handle, _lib.DF_THETA_GIVEN))
    np.testing.assert_array_equal(grad(tr, thn), g_given)  # GIVEN ignores the bounds
    _lib.check(tr.lib.df_train_set_theta_input(tr.handle, _lib.DF_THETA_RAW))
    np.testing.assert_array_equal(grad(tr, th), g_given)
    assert tr.lib.df_train_set_theta_input(tr.handle, 7) == _lib.DF_ERR_INVALID
    # RAW without bounds is refused
    h2 = spec_to_chain(spec)
    tr2 = HIPTrainer(h2, Adam())
    _lib.check(tr2.lib.df_train_set_theta_input(tr2.handle, _lib.DF_THETA_RAW))
    with pytest.raises(_lib.ArgumentError):
        grad(tr2, th)

    # graph steps: captured under AUTO without bounds (θ as given), then bounds set —
    # the replay must switch to normalising (the parameters then match an eager twin)
    a = HIPTrainer(spec_to_chain(spec), Adam())
    b = HIPTrainer(spec_to_chain(spec), Adam())
    xb, tb = _dev(x, cuda), _dev(thn, cuda)
    tb_raw = _dev(th, cuda)
    for _ in range(3):                                    # eager, capture, replay
        a.step_graph(xb, tb, 512)
        b.step(xb, tb, 512)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.get_params(), b.get_params())
    a.chain.set_theta_bounds(tmin, tmax)
    b.chain.set_theta_bounds(tmin, tmax)
    tb.copy_(tb_raw)                                      # same buffer, raw θ now
    for _ in range(3):
        a.step_graph(xb, tb, 512)
        b.step(xb, tb, 512)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.get_params(), b.get_params())
    # new bounds under the same convention (AUTO, bounds set before
    # and after) keep the capture; its replays must read the NEW bounds in every kernel
    # (the small-batch inverse pass included: batch 512 of the README chain runs on it)
    tmin2, tmax2 = np.array([-3.0], np.float32), np.array([0.5], np.float32)
    a.chain.set_theta_bounds(tmin2, tmax2)
    b.chain.set_theta_bounds(tmin2, tmax2)
    for _ in range(3):
        a.step_graph(xb, tb, 512)
        b.step(xb, tb, 512)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.get_params(), b.get_params())


def spec_to_chain(spec):
    from helpers import spec_to_element

    return spec_to_element(spec).hip()
