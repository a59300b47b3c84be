"""Host-side logic on CPU: the C-ABI library loads and exports every symbol the
header declares; descriptors are validated/planned without a device; the
Python mirror reproduces the reference's index tables bit for bit."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import densityflows_amd as dfa
from densityflows_amd import _lib, hip
from helpers import spec_to_element
from oracle import flow_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "densityflows_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(df_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), "ctypes signatures out of sync with the header"
    assert lib.df_get_abi_version() == _lib.ABI_VERSION


def test_limits():
    lim = _lib.df_limits()
    _lib.check(_lib.load().df_get_limits(C.byref(lim)))
    assert lim.max_state == 64 and lim.max_hidden == 256 and lim.max_af == 32


def test_plan_config2_and_config1():
    rng = np.random.default_rng(0)
    ch2 = dfa.FlowChain.repeat(dfa.CouplingBlock, 4, 5, hidden_dim_s=64, hidden_dim_t=64, rng=rng)
    info = hip.validate(ch2.layers)
    assert info.n_params == 72744 and info.flops_per_sample == 141312.0
    assert info.hidden_tiles == 4
    x = np.load(os.path.join(ROOT, "tests", "golden", "datatest_x.npy"))
    th = np.load(os.path.join(ROOT, "tests", "golden", "datatest_theta.npy"))
    data = dfa.DataArrays(x, th, rng=rng)
    ch1 = dfa.FlowChain(*[dfa.CouplingLayer(data, m, hidden_dim_s=16, hidden_dim_t=16, rng=rng)
                          for m in ([1, 2, 3], [3, 4, 5], [5, 1, 2])],
                        dfa.NormalizationLayer.from_data(x, -1.0, 1.0))
    info = hip.validate(ch1.layers)
    assert info.n_params == 2322 and info.flops_per_sample == 4224.0 and info.n_stages == 1


@pytest.mark.parametrize("exact", ["0", "1"])
def test_plan_kernel_choice_split(monkeypatch, exact):
    """Config 2 plans the FAST SPLIT kernel (id 4), config 4 the wide SPLIT kernel
    (id 6), config 1 (hidden 16) the exact FAST kernel (id 3); DF_F32_EXACT=1 plans
    the exact-f32 kernels.  split_flops_per_sample is the FLOP the SPLIT kernels run
    as bf16x3 products: first + hidden Dense of every net at config 2, all three
    Denses at config 4."""
    monkeypatch.setenv("DF_F32_EXACT", exact)
    rng = np.random.default_rng(0)
    ch2 = dfa.FlowChain.repeat(dfa.CouplingBlock, 4, 5, hidden_dim_s=64, hidden_dim_t=64, rng=rng)
    i2 = hip.validate(ch2.layers)
    ch4 = dfa.FlowChain.repeat(dfa.CouplingBlock, 8, 32, n=8, hidden_dim_s=256, hidden_dim_t=256, rng=rng)
    i4 = hip.validate(ch4.layers)
    ch1 = dfa.FlowChain.repeat(dfa.CouplingBlock, 2, 5, hidden_dim_s=16, hidden_dim_t=16, rng=rng)
    i1 = hip.validate(ch1.layers)
    if exact == "1":
        assert (i2.kernel, i4.kernel, i1.kernel) == (3, 5, 3)
        assert i2.split_flops_per_sample == i4.split_flops_per_sample == 0.0
    else:
        assert (i2.kernel, i4.kernel, i1.kernel) == (4, 6, 3)
        # per net 2·(in·64 + 64·64), in = 2 or 3 (the 64·out output GEMV stays f32)
        want2 = sum(2.0 * (inn * 64 + 64 * 64) for inn in (2, 3) * 4 for _net in (0, 1))
        assert i2.split_flops_per_sample == want2
        assert i4.split_flops_per_sample == i4.flops_per_sample


def _bf16_rne(v):
    """f32 → bf16 bits by round-to-nearest-even (df_plan.h bf16_rne_bits), as f32."""
    u = np.asarray(v, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def test_bf16x3_split_is_exact_and_six_products_are_f32_accurate():
    """The SPLIT arithmetic, restated in numpy: three RNE bf16 planes
    sum exactly to the f32 value, and the six kept products w0x0 + w0x1 + w1x0 +
    w0x2 + w1x1 + w2x0 (each exact in f32) differ from w·x by less than 2^-24·|w·x|."""
    rng = np.random.default_rng(5)
    w = (rng.standard_normal(200000) * np.exp(rng.uniform(-20, 20, 200000))).astype(np.float32)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-20, 20, 200000))).astype(np.float32)

    def planes(a):
        p0 = _bf16_rne(a)
        r = (a - p0).astype(np.float32)
        p1 = _bf16_rne(r)
        p2 = _bf16_rne((r - p1).astype(np.float32))
        return p0, p1, p2

    w0, w1, w2 = planes(w)
    x0, x1, x2 = planes(x)
    for a, (a0, a1, a2) in ((w, (w0, w1, w2)), (x, (x0, x1, x2))):
        np.testing.assert_array_equal(a0.astype(np.float64) + a1 + a2, a.astype(np.float64))
    d = np.float64
    six = (w0.astype(d) * x0 + w0.astype(d) * x1 + w1.astype(d) * x0 + w0.astype(d) * x2
           + w1.astype(d) * x1 + w2.astype(d) * x0)
    exact = w.astype(d) * x.astype(d)
    rel = np.abs(six - exact) / np.abs(exact)
    assert rel.max() < 2.0 ** -24, rel.max()
    # every bf16 product is exact in f32 (8 + 8 significand bits)
    for a, b in ((w0, x0), (w0, x1), (w2, x0)):
        p = a.astype(d) * b.astype(d)
        np.testing.assert_array_equal(p.astype(np.float32).astype(d), p)


def test_plan_config4():
    rng = np.random.default_rng(0)
    ch4 = dfa.FlowChain.repeat(dfa.CouplingBlock, 8, 32, n=8, hidden_dim_s=256, hidden_dim_t=256, rng=rng)
    info = hip.validate(ch4.layers)
    assert info.n_params == 2441728 and info.flops_per_sample == 4849664.0
    assert info.hidden_tiles == 16 and info.n_stages > 16


def test_doctest_summaries():
    # src/Layers.jl:99-104 and src/Blocks.jl:51-59
    s = dfa.summarize(dfa.CouplingLayer(3, [1, 3], n=2, hidden_dim=10, n_sublayers_s=1, σ="tanh"))
    assert s.splitlines() == [
        "RNVPCouplingLayer | s_net > [3, 10, 2] (62 parameters)",
        "                  | t_net > [3, 10, 10, 2] (172 parameters)",
        "                  | axes  > (d,n)=(3,2); identity=(2), transformed=(1,3)"]
    b = dfa.summarize(dfa.CouplingBlock.build(3, [1, 3], n=2, hidden_dim=10, n_sublayers_s=1, σ="tanh"))
    assert b.splitlines()[3:] == [
        "RNVPCouplingLayer | s_net > [4, 10, 1] (61 parameters)",
        "                  | t_net > [4, 10, 10, 1] (171 parameters)",
        "                  | axes  > (d,n)=(3,2); identity=(1,3), transformed=(2)"]


@pytest.mark.parametrize("mask", [[1, 2, 3], [5, 1, 2], [4, 2, 5, 1, 6], [3]])
def test_axes_tables_match_oracle(mask):
    d = max(6, max(mask))
    a = dfa.CouplingAxes.from_mask(d, mask, n=2)
    o = O.coupling_axes(d, mask, n=2)
    assert (a.axis_id, a.axis_af, a.axis_nn) == (o["axis_id"], o["axis_af"], o["axis_nn"])
    r, ro = dfa.reverse(a), O.reverse_axes(o)
    assert (r.axis_id, r.axis_af, r.axis_nn) == (ro["axis_id"], ro["axis_af"], ro["axis_nn"])
    assert dfa.is_reverse(a, r)


def test_axes_equality_runtests():
    data = dfa.DataArrays(np.ones((7, 10), np.float32), np.ones((2, 10), np.float32))
    from densityflows_amd.axes import CouplingAxes_
    ref = dfa.CouplingAxes.from_cut(7, 3, n=2)
    assert dfa.CouplingAxes.from_mask(7, [4, 5, 6, 7], n=2) == ref
    assert CouplingAxes_(data) == ref
    assert CouplingAxes_(data, [4, 5, 6, 7]) == ref
    assert CouplingAxes_(data, 3) == ref


def test_spec_roundtrip():
    rng = np.random.default_rng(1)
    ch = dfa.FlowChain(dfa.CouplingLayer(5, [2, 4], n=1, rng=rng), dfa.CouplingBlock.build(5, 2, n=1, rng=rng))
    again = spec_to_element(ch.to_spec())
    assert again.num_params() == ch.num_params()
    np.testing.assert_array_equal(again[0].s_net[0].W, ch[0].s_net[0].W)


def test_validation_errors_map_to_reference_exceptions():
    rng = np.random.default_rng(2)
    # NormalizationLayer β ≤ α  (Normalization.jl:55)
    with pytest.raises(AssertionError):
        dfa.NormalizationLayer(np.zeros(3), np.ones(3), 1.0, 0.0)
    # CouplingBlock with non-complementary axes (Blocks.jl:71)
    l1 = dfa.CouplingLayer(5, [1, 2], rng=rng)
    l2 = dfa.CouplingLayer(5, [3, 4], rng=rng)
    with pytest.raises(dfa.ArgumentError):
        dfa.CouplingBlock(l1, l2)
    # mask beyond d (Axes.jl:85)
    with pytest.raises(AssertionError):
        dfa.CouplingAxes.from_mask(3, [4])
    # mixed d in one chain
    with pytest.raises(AssertionError):
        hip.validate([dfa.CouplingLayer(5, [1], rng=rng), dfa.CouplingLayer(6, [1], rng=rng)])
    # hidden width beyond the kernel limit
    with pytest.raises(dfa.UnsupportedError):
        hip.validate([dfa.CouplingLayer(5, [1], hidden_dim=300, rng=rng)])


def test_c_abi_rejects_bad_descriptor_without_device():
    lib = _lib.load()
    desc = _lib.df_chain_desc(_lib.ABI_VERSION + 7, 5, 0, 0, None)
    assert lib.df_chain_validate(C.byref(desc), None) == _lib.DF_ERR_INVALID
    assert b"ABI" in lib.df_last_error()
    desc = _lib.df_chain_desc(_lib.ABI_VERSION, 70, 0, 1, None)
    assert lib.df_chain_validate(C.byref(desc), None) == _lib.DF_ERR_UNSUPPORTED


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "densityflows.jl_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h", ".jl")):
                src = open(os.path.join(dirpath, f), encoding="utf-8").read()
                assert "flow_oracle" not in src and "oracle/" not in src, f


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    rng = np.random.default_rng(3)
    ch = dfa.FlowChain(dfa.CouplingLayer(5, [1, 2], rng=rng))
    with pytest.raises(dfa.HIPError):
        dfa.forward(ch, np.zeros((5, 4), np.float32))


def test_comm_entry_points_fail_cleanly_without_a_device():
    """df_comm_* are exported and argument-checked on a host without a GPU (the
    RCCL calls themselves need one: tests/test_gpu_comm.py)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("host-only check")
    lib = _lib.load()
    h = C.c_void_p()
    uid = C.create_string_buffer(_lib.DF_COMM_ID_BYTES)
    assert lib.df_comm_init_rank(C.byref(h), 1, uid, 0, 0) != _lib.DF_OK and not h.value
    assert lib.df_comm_init_rank(C.byref(h), 2, uid, 2, 0) == _lib.DF_ERR_INVALID   # rank out of range
    assert lib.df_comm_destroy(None) == _lib.DF_OK
    assert lib.df_comm_allreduce_sum(None, None, 4, _lib.DF_DTYPE_F32, None) == _lib.DF_ERR_INVALID
    assert lib.df_flow_nll(None, None, None, None, 4, None, None) == _lib.DF_ERR_INVALID
    assert lib.df_train_set_debug(None, 1) == _lib.DF_ERR_INVALID
    assert lib.df_chain_set_weights(None, None) == _lib.DF_ERR_INVALID


def test_julia_shim_binds_only_declared_symbols():
    """The Julia ccall shim (never executed here: no Julia toolchain)
    names only entry points include/densityflows_hip.h declares, with balanced
    blocks, and covers the ABI's groups (chain passes, flow NLL, training, RCCL)."""
    import re

    src = open(os.path.join(ROOT, "densityflows.jl_amd", "julia", "DensityFlowsHIP.jl")).read()
    hdr = open(os.path.join(ROOT, "include", "densityflows_hip.h")).read()
    declared = set(re.findall(r"\b(df_[a-z0-9_]+)\s*\(", hdr))
    called = set(re.findall(r"ccall\(\(:?\(?:?(df_[a-z0-9_]+)", src)) | set(re.findall(r":(df_[a-z0-9_]+)", src))
    assert called, "no ccall found"
    assert called <= declared, sorted(called - declared)
    for sym in ("df_chain_forward_inplace", "df_chain_logpdf_sum", "df_chain_nll", "df_train_step",
                "df_train_step_dist", "df_train_set_debug", "df_comm_init_rank", "df_comm_get_unique_id"):
        assert sym in called, sym
    # block balance: every opener (function/struct/if/for/try/begin/do/let/module) has an `end`
    code = re.sub(r'""".*?"""', "", src, flags=re.S)
    code = re.sub(r"#=.*?=#", "", code, flags=re.S)
    code = re.sub(r"#.*", "", code)
    code = re.sub(r'"(\\.|[^"\\])*"', '""', code)
    opens = len(re.findall(r"^\s*(?:mutable struct|struct|function|module|if|for|while|try|let|begin)\b",
                           code, flags=re.M))
    opens += len(re.findall(r"\bdo\b(?:\s+\w+)?\s*$", code, flags=re.M))
    opens += len(re.findall(r"\bbegin\s*$", code, flags=re.M)) - len(re.findall(r"^\s*begin\s*$", code, flags=re.M))
    ends = len(re.findall(r"(?<![:\[])\bend\b(?!\s*\])", code))  # not an index `a[2:end]`
    assert opens == ends, (opens, ends)
