"""Replay of the Julia front-end's C-call sequences through ctypes (test infrastructure).

There is no Julia toolchain in this pipeline, so the host logic of
densityflows.jl_amd/julia/DensityFlowsHIP.jl cannot run.  This module re-enacts it,
function for function: each function below issues the same ccalls, in the same
order, with the same arguments (device buffers from df_device_alloc, copies through
df_memcpy_h2d / df_memcpy_d2h, the NULL stream, staging slots grown on demand) as the
Julia function it is named after (`!` spelled `_bang`).  Host-side Julia semantics
that decide what reaches the library are restated too: `normalized_training_data`
(src/Data.jl:189-199), `Flux.DataLoader` without shuffling (contiguous batches, the
partial last batch kept), the Float32 / Float64 conversions of the losses.

  * tests/test_julia_shim.py checks statically that every function here issues the
    same ccall symbols, in the same order, as its Julia counterpart;
  * tests/test_gpu_julia_replay.py runs the replay (sample → train! → sample) against
    the oracle's epoch loop.

Every library call goes through `cc`, which records the symbol in `CALLS`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from densityflows_amd import _lib
from densityflows_amd.hip import _Desc, chain_dims, flatten_elements
from densityflows_amd.train import _dense_order
from densityflows_amd.train import trainables as _flux_trainables

CALLS: list = []
_L = None


def lib():
    global _L
    if _L is None:
        _L = _lib.load()
    return _L


def cc(sym: str, *args):
    """One ccall((:sym, LIB), ...) of the shim."""
    CALLS.append(sym)
    return getattr(lib(), sym)(*args)


NULL = C.c_void_p(0)
DF_ERR_NONFINITE = -6
DF_THETA_GIVEN = 2


class NonFiniteLoss(Exception):
    def __init__(self, loss):
        super().__init__(f"non-finite loss {loss}")
        self.loss = loss


# ---- errors (DensityFlowsHIP.jl: lasterror, check) -----------------------------------
def lasterror():
    return cc("df_last_error").decode("utf-8", "replace")


def check(rc, what):
    if rc == 0:
        return None
    msg = f"{what}: " + lasterror()
    if rc == -1:
        raise _lib.ArgumentError(msg)
    if rc == -2:
        raise _lib.DimensionMismatch(msg)
    raise RuntimeError(f"densityflows_hip [{rc}] {msg}")


def __init__():
    v = cc("df_get_abi_version")
    assert v == _lib.ABI_VERSION, f"library ABI {v}, binding {_lib.ABI_VERSION}"


# ---- staging (Staging, _buf!, _release!) ----------------------------------------------
class Staging:
    def __init__(self, n):
        self.ptr = [None] * n
        self.bytes = [0] * n


def _buf_bang(st, i, nbytes):
    i -= 1  # Julia's 1-based slot
    if st.bytes[i] < nbytes:
        if st.ptr[i] is not None:
            _free(st.ptr[i])
        st.ptr[i] = None
        st.bytes[i] = 0
        st.ptr[i] = _dev(nbytes)
        st.bytes[i] = max(nbytes, 1)
    return st.ptr[i]


def _release_bang(st):
    for p in st.ptr:
        if p is not None:
            _free(p)
    st.ptr = [None] * len(st.ptr)
    st.bytes = [0] * len(st.bytes)


# ---- device memory helpers (_dev, _free, _h2d, _d2h) ---------------------------------
def _dev(nbytes):
    p = C.c_void_p()
    check(cc("df_device_alloc", C.byref(p), max(nbytes, 1)), "df_device_alloc")
    return p


def _free(p):
    return cc("df_device_free", p)


def _h2d(dst, src: np.ndarray):
    check(cc("df_memcpy_h2d", dst, src.ctypes.data_as(C.c_void_p), src.nbytes, NULL), "h2d")


def _d2h(dst: np.ndarray, src):
    check(cc("df_memcpy_d2h", dst.ctypes.data_as(C.c_void_p), src, dst.nbytes, NULL), "d2h")


def _dense(a):
    """Array{Float32} of a (possibly strided) view, Julia memory order: column-major."""
    return np.asfortranarray(np.asarray(a, np.float32))


def _sizeof(a):
    return a.nbytes


# ---- the chain handle (HIPFlowChain) -------------------------------------------------
class _Chain:
    pass


def HIPFlowChain(chain, device=0):
    """HIPFlowChain(chain::FlowChain; device): df_chain_create from the flattened layers."""
    flat = flatten_elements(chain.layers)
    d, n = chain_dims(flat)
    desc = _Desc(flat, d, n)
    h = C.c_void_p()
    check(cc("df_chain_create", C.byref(h), C.byref(desc.desc), device), "df_chain_create")
    params = _flux_trainables(chain).astype(np.float32)
    obj = _Chain()
    obj.handle, obj.d, obj.n = h, d, max(n, 0)
    obj.stage = Staging(5)
    obj.params = params
    obj.trainer = None
    obj.trainer_key = None
    obj.bounds = None

    def fin(c):
        _release_bang(c.stage)
        if c.trainer is not None:
            _destroy_bang(c.trainer)
        cc("df_chain_destroy", c.handle)

    obj.finalize = lambda: fin(obj)
    return obj


def _run(sym, c, y, th):
    y, th = _dense(y), _dense(th)
    assert y.shape[0] == c.d, "input must be (d, dims...)"
    assert th.shape[0] == c.n, "dimensions θ must match (n, dims...) with n number of trained parameters"
    B = int(np.prod(y.shape[1:]))
    out = np.empty_like(y, order="F")
    ldj = np.empty(y.shape[1:], np.float32, order="F")
    dy, dth = _buf_bang(c.stage, 1, _sizeof(y)), _buf_bang(c.stage, 2, _sizeof(th))
    dout, dl = _buf_bang(c.stage, 3, _sizeof(y)), _buf_bang(c.stage, 4, _sizeof(ldj))
    _h2d(dy, y)
    if c.n > 0:
        _h2d(dth, th)
    check(cc(sym, c.handle, dy, dth if c.n > 0 else NULL, dout, dl, C.c_int64(B), NULL), sym)
    _d2h(out, dout)
    _d2h(ldj, dl)
    return out, ldj


def forward(c, z, th):
    return _run("df_chain_forward", c, z, th)


def backward(c, x, th):
    return _run("df_chain_backward", c, x, th)


def forward_bang(c, z, th):
    zz, th = _dense(z), _dense(th)
    B = int(np.prod(z.shape[1:]))
    dz, dth = _buf_bang(c.stage, 1, _sizeof(zz)), _buf_bang(c.stage, 2, _sizeof(th))
    _h2d(dz, zz)
    if c.n > 0:
        _h2d(dth, th)
    check(cc("df_chain_forward_inplace", c.handle, dz, dth if c.n > 0 else NULL, C.c_int64(B), NULL),
          "df_chain_forward_inplace")
    _d2h(zz, dz)
    z[...] = zz
    return None


def logpdf_sum(c, x, th):
    x, th = _dense(x), _dense(th)
    B = int(np.prod(x.shape[1:]))
    dx, dth, ds = _buf_bang(c.stage, 1, _sizeof(x)), _buf_bang(c.stage, 2, _sizeof(th)), _buf_bang(c.stage, 5, 16)
    _h2d(dx, x)
    if c.n > 0:
        _h2d(dth, th)
    check(cc("df_chain_logpdf_sum", c.handle, dx, dth if c.n > 0 else NULL, ds, C.c_int64(B), NULL),
          "df_chain_logpdf_sum")
    r = np.empty(1, np.float64)
    _d2h(r, ds)
    return float(r[0])


# ---- training (HIPTrainer, train_step!, trainables, set_debug!) ----------------------
class _Trainer:
    pass


def _destroy_bang(t):
    if t.handle is None:
        return None
    _release_bang(t.stage)
    cc("df_train_destroy", t.handle)
    t.handle = None
    return None


def HIPTrainer(c, eta=1e-3, beta=(0.9, 0.999), epsilon=1e-8):
    t = C.c_void_p()
    check(cc("df_train_create", C.byref(t), c.handle, C.byref(_lib.df_adam(eta, beta[0], beta[1], epsilon))),
          "df_train_create")
    n = C.c_int64()
    check(cc("df_train_num_params", t, C.byref(n)), "df_train_num_params")
    check(cc("df_train_set_theta_input", t, DF_THETA_GIVEN), "df_train_set_theta_input")
    obj = _Trainer()
    obj.handle, obj.chain, obj.n_params, obj.stage = t, c, int(n.value), Staging(3)
    return obj


def train_step_bang(t, x, th):
    x, th = _dense(x), _dense(th)
    B = int(np.prod(x.shape[1:]))
    dx, dth, ds = _buf_bang(t.stage, 1, _sizeof(x)), _buf_bang(t.stage, 2, _sizeof(th)), _buf_bang(t.stage, 3, 8)
    _h2d(dx, x)
    if t.chain.n > 0:
        _h2d(dth, th)
    rc = cc("df_train_step", t.handle, dx, dth if t.chain.n > 0 else NULL, C.c_int64(B), ds, NULL)
    r = np.empty(1, np.float64)
    if rc != DF_ERR_NONFINITE:
        check(rc, "df_train_step")
    _d2h(r, ds)
    loss = np.float32(-r[0] / B)
    if rc == DF_ERR_NONFINITE:
        raise NonFiniteLoss(loss)
    return loss


def trainables(t):
    p = np.empty(t.n_params, np.float32)
    check(cc("df_train_get_params", t.handle, p.ctypes.data_as(C.POINTER(C.c_float)), C.c_int64(t.n_params)),
          "df_train_get_params")
    return p


def set_debug_bang(t, on):
    check(cc("df_train_set_debug", t.handle, 1 if on else 0), "df_train_set_debug")


def _trainer_bang(c, rule):
    key = (np.float32(rule.eta), (np.float32(rule.beta[0]), np.float32(rule.beta[1])), np.float32(rule.epsilon))
    if c.trainer is None or c.trainer_key != key:
        if c.trainer is not None:
            _destroy_bang(c.trainer)
        c.trainer = HIPTrainer(c, eta=rule.eta, beta=rule.beta, epsilon=rule.epsilon)
        c.trainer_key = key
    return c.trainer


# ---- train! (_hip_train!) ------------------------------------------------------------
class Flow:
    """The fields of DensityFlows.Flow that _hip_train! / _hip_sample read."""

    def __init__(self, c, metadata):
        self.model = [c]            # FlowChain((HIPFlowChain(chain),)).layers
        self.metadata = metadata
        self.train_loss = []
        self.valid_loss = []


def normalize_input(x, x_min, x_max):
    """src/Data.jl:213-218 in Float32: (x .- x_min) ./ x_diff, rows with x_diff == 0 set to 0."""
    x = np.asarray(x, np.float32)
    x_min = np.asarray(x_min, np.float32).reshape(-1, 1)
    x_diff = np.asarray(x_max, np.float32).reshape(-1, 1) - x_min
    with np.errstate(divide="ignore", invalid="ignore"):
        y = (x - x_min) / x_diff
    y[(x_diff == 0).ravel(), :] = 0
    return y


def normalized_data(data, md, which):
    x, th = data.training_data() if which == "training" else data.validation_data()
    return x, normalize_input(th, md.theta_min, md.theta_max)


def _data_loader(xy, batchsize):
    """Flux.DataLoader(data; batchsize, shuffle=false): contiguous batches, last partial kept."""
    x, th = xy
    N = x.shape[1]
    for b0 in range(0, N, batchsize):
        yield x[:, b0:b0 + batchsize], th[:, b0:b0 + batchsize]


def _hip_train_bang(flow, data, t, epochs=100, batchsize=64, shuffle=False, verbose=True, debug=False):
    if shuffle:
        raise NotImplementedError("the replay has no Julia RNG: shuffle=false only")
    c = flow.model[0]
    set_debug_bang(t, debug)
    train_data = normalized_data(data, flow.metadata, "training")
    valid_data = normalized_data(data, flow.metadata, "validation")

    def setloss(s):
        return np.float32(-logpdf_sum(c, *s) / int(np.prod(s[0].shape[1:])))

    for _ in range(epochs):
        for x_batch, t_batch in _data_loader(train_data, batchsize):
            try:
                train_step_bang(t, x_batch, t_batch)
            except NonFiniteLoss as e:
                c.params[:] = trainables(t)
                z, ldj = backward(c, x_batch, t_batch)
                print(f"{e.loss}, {ldj}, {z}")
                raise _lib.ArgumentError("") from e
        train_loss = setloss(train_data)
        flow.train_loss.append(train_loss)
        if debug and not np.isfinite(train_loss):
            print(f"Problem with train loss {train_loss}")
            c.params[:] = trainables(t)
            return backward(c, *train_data)
        valid_loss = setloss(valid_data)
        flow.valid_loss.append(valid_loss)
        if debug and not np.isfinite(valid_loss):
            print(f"Problem with valid loss {valid_loss}")
            c.params[:] = trainables(t)
            return backward(c, *valid_data)
        if verbose:
            print(f"epoch: {len(flow.train_loss)} | train_loss = {train_loss}, valid_loss = {valid_loss}")
    c.params[:] = trainables(t)
    return (None, None) if debug else None


def train_bang(flow, data, rule, **kws):
    """train!(flow, data, Optimisers.setup(rule, flow.model)) → _hip_train!(flow, data, _trainer!(c, rule))."""
    return _hip_train_bang(flow, data, _trainer_bang(flow.model[0], rule), **kws)


# ---- sample (_set_bounds!, _hip_sample) ----------------------------------------------
def _set_bounds_bang(c, md):
    if c.n == 0:
        return None
    b = (np.ascontiguousarray(md.theta_min, np.float32), np.ascontiguousarray(md.theta_max, np.float32))
    if c.bounds is not None and all(np.array_equal(u, v) for u, v in zip(c.bounds, b)):
        return None
    check(cc("df_chain_set_theta_bounds", c.handle, b[0].ctypes.data_as(C.POINTER(C.c_float)),
             b[1].ctypes.data_as(C.POINTER(C.c_float))), "df_chain_set_theta_bounds")
    c.bounds = b
    return None


def _hip_sample(seed, flow, dims, th, bcast):
    """`rand(rng, UInt64)` of the Julia method is the explicit `seed` here."""
    c = flow.model[0]
    _set_bounds_bang(c, flow.metadata)
    B = int(np.prod(dims))
    r = np.empty((c.d,) + tuple(dims), np.float32, order="F")
    th = _dense(th)
    dr, dth = _buf_bang(c.stage, 3, _sizeof(r)), _buf_bang(c.stage, 2, _sizeof(th))
    if c.n > 0:
        _h2d(dth, th)
    check(cc("df_flow_sample", c.handle, dr, dth if c.n > 0 else NULL, 1 if bcast else 0, C.c_int64(B),
             C.c_uint64(seed), C.c_uint64(0), NULL), "df_flow_sample")
    _d2h(r, dr)
    return r


def train_step_graph_bang(t, x_ptr, th_ptr, B, stream=NULL):
    check(cc("df_train_step_graph", t.handle, x_ptr, th_ptr, C.c_int64(B), C.c_int64(B), NULL, stream),
          "df_train_step_graph")
    return None


# ---- weight export (copy_trainables!) ------------------------------------------------------
def _flux_trainables_arrays(model):
    """Flux.trainables(model) of the Python mirror: the arrays in the order Functors walks
    them (FlowChain elements; per coupling layer s_net then t_net, trainable=(s_net,
    t_net) in src/affine/RNVP.jl:51, NICE t_net only, NormalizationLayer none; per Dense
    weight then bias), each as (Dense, field name)."""
    for D in _dense_order(model.layers):
        yield D, "W"
        if D.b is not None:
            yield D, "b"


def copy_trainables_bang(model, p):
    """copy_trainables!(model, p): `copyto!(a, 1, p, off + 1, n)` into each trainable array
    (a Julia array fills column-major), then the length check."""
    p = np.asarray(p, np.float32)
    off = 0
    for D, name in _flux_trainables_arrays(model):
        a = getattr(D, name)
        n = a.size
        if off + n > len(p):  # copyto! past the end of p: Julia's BoundsError
            raise IndexError(f"copyto!: {n} elements from offset {off + 1} of a vector of length {len(p)}")
        setattr(D, name, p[off:off + n].reshape(a.shape, order="F").copy())
        off += n
    if off != len(p):
        raise _lib.DimensionMismatch(f"model has {off} trainables, device vector {len(p)}")
    return model


# ---- multi-GPU (comm_unique_id, HIPComm, flow_nll, train_step_dist!) ---------------------
class _Comm:
    pass


def comm_unique_id():
    uid = (C.c_uint8 * 128)()
    check(cc("df_comm_get_unique_id", uid), "df_comm_get_unique_id")
    return uid


def HIPComm(nranks, uid, rank, device=0):
    h = C.c_void_p()
    check(cc("df_comm_init_rank", C.byref(h), nranks, uid, rank, device), "df_comm_init_rank")
    obj = _Comm()
    obj.handle, obj.rank, obj.nranks, obj.stage = h, rank, nranks, Staging(1)

    def fin(c):
        _release_bang(c.stage)
        cc("df_comm_destroy", c.handle)

    obj.finalize = lambda: fin(obj)
    return obj


def flow_nll(c, comm, x, th):
    x, th = _dense(x), _dense(th)
    B = int(np.prod(x.shape[1:]))
    dx, dth, ds = _buf_bang(c.stage, 1, _sizeof(x)), _buf_bang(c.stage, 2, _sizeof(th)), _buf_bang(c.stage, 5, 16)
    _h2d(dx, x)
    if c.n > 0:
        _h2d(dth, th)
    check(cc("df_chain_nll", c.handle, NULL if comm is None else comm.handle, dx, dth if c.n > 0 else NULL,
             C.c_int64(B), ds, NULL), "df_chain_nll")
    r = np.empty(2, np.float64)
    _d2h(r, ds)
    return np.float32(-r[0] / r[1])


def train_step_dist_bang(t, comm, x, th, n_total):
    x, th = _dense(x), _dense(th)
    B = int(np.prod(x.shape[1:]))
    dx, dth, ds = _buf_bang(t.stage, 1, _sizeof(x)), _buf_bang(t.stage, 2, _sizeof(th)), _buf_bang(t.stage, 3, 8)
    _h2d(dx, x)
    if t.chain.n > 0:
        _h2d(dth, th)
    rc = cc("df_train_step_dist", t.handle, comm.handle if comm is not None else NULL, dx,
            dth if t.chain.n > 0 else NULL, C.c_int64(B), C.c_int64(n_total), ds, NULL)
    if rc != DF_ERR_NONFINITE:
        check(rc, "df_train_step_dist")
    r = np.empty(1, np.float64)
    _d2h(r, ds)
    loss = np.float32(-r[0] / n_total)
    if rc == DF_ERR_NONFINITE:
        raise NonFiniteLoss(loss)
    return loss
