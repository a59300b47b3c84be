"""Training — mirror of ``train!`` (src/Flows.jl:380-445) with Optimisers.Adam.

Every step runs on the device through the C ABI (``df_train_*``): the fused
inverse pass keeps each layer's output, the reverse sweep recomputes the
s/t conditioners and back-propagates through the coupling pullbacks
(``rrule(RNVP_backward)`` src/affine/RNVP.jl:99-147, ``rrule(NICE_backward)``
src/affine/NICE.jl:84-113) and the Dense chains on MFMA, gradients are
reduced in a fixed order, then Adam updates the flat parameters and the
packed weights are regathered, so the Flow's forward / logpdf / sample see
the new parameters immediately.

Data parallelism (one process per GPU): :func:`train_` with a
``torch.distributed`` process group shards every batch over the ranks,
computes per-rank gradients with the mean taken over the global batch, and
all-reduces the flat gradient (RCCL over xGMI with the ``nccl`` backend)
before the identical Adam step on every rank.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from .hip import HIPChain, _ptr, _stream, as_julia_device, flatten_elements
from .layers import NormalizationLayer, RNVPCouplingLayer

__all__ = ["Adam", "setup", "TrainState", "HIPTrainer", "train_", "trainables", "load_trainables"]


class Adam:
    """``Optimisers.Adam(η = 1f-3, β = (9f-1, 9.99f-1), ϵ = 1f-8)``."""

    def __init__(self, eta: float = 1e-3, beta=(0.9, 0.999), epsilon: float = 1e-8):
        self.eta = float(eta)
        self.beta = (float(beta[0]), float(beta[1]))
        self.epsilon = float(epsilon)

    def __repr__(self):
        return f"Adam(eta={self.eta}, beta={self.beta}, epsilon={self.epsilon})"


class _DeviceArray:
    """A raw device float32 vector exposed to torch via __cuda_array_interface__."""

    def __init__(self, ptr: int, count: int):
        self.__cuda_array_interface__ = {"shape": (int(count),), "typestr": "<f4", "data": (int(ptr), False),
                                         "version": 2, "strides": None}


# reverse-sweep forms (df_sweep_form, include/densityflows_hip.h)
SWEEP_AUTO, SWEEP_FUSED, SWEEP_H0FREE, SWEEP_KEPT, SWEEP_RECOMPUTE, SWEEP_LAYERWISE = 0, 1, 2, 3, 4, 5
SWEEP_SEPARATE = 16
# the form a HIPTrainer requests when none is given (tests set it to exercise one path
# through code that builds its own trainers, e.g. train_)
DEFAULT_SWEEP = SWEEP_AUTO
SWEEP_NAMES = {SWEEP_FUSED: "fused", SWEEP_H0FREE: "h0free", SWEEP_KEPT: "kept", SWEEP_RECOMPUTE: "recompute"}


class HIPTrainer:
    """A ``df_train`` handle bound to a compiled chain (one device).  ``sweep``: a
    df_sweep_form to request (default: the library picks, SWEEP_AUTO)."""

    def __init__(self, chain: HIPChain, opt: Adam, sweep: int | None = None):
        self.chain = chain  # keeps the df_chain alive for this handle's lifetime
        self.lib = chain.lib
        self.opt = opt
        h = C.c_void_p()
        a = _lib.df_adam(opt.eta, opt.beta[0], opt.beta[1], opt.epsilon)
        sweep = DEFAULT_SWEEP if sweep is None else sweep
        if sweep == SWEEP_AUTO and not hasattr(self.lib, "df_train_create_ex"):  # a pre-ABI-5 build (A/B runs)
            _lib.check(self.lib.df_train_create(C.byref(h), chain.handle, C.byref(a)), "df_train_create")
        else:
            _lib.check(self.lib.df_train_create_ex(C.byref(h), chain.handle, C.byref(a), int(sweep)),
                       "df_train_create_ex")
        self.handle = h
        n = C.c_int64()
        _lib.check(self.lib.df_train_num_params(self.handle, C.byref(n)))
        self.num_params = int(n.value)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.df_train_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None

    @property
    def device(self):
        return self.chain.device

    def grad(self):
        """The flat gradient as a torch tensor aliasing the device buffer."""
        import torch

        p = C.c_void_p()
        _lib.check(self.lib.df_train_grad_ptr(self.handle, C.byref(p)))
        return torch.as_tensor(_DeviceArray(p.value or 0, self.num_params), device=self.device)

    def gradient(self, xbuf, thbuf, batch: int, n_total: int, lpsum=None):
        _lib.check(self.lib.df_train_gradient(self.handle, _ptr(xbuf), _ptr(thbuf), C.c_int64(batch),
                                              C.c_int64(n_total), _ptr(lpsum), _stream(self.device)),
                   "df_train_gradient")

    def apply(self):
        _lib.check(self.lib.df_train_apply(self.handle, _stream(self.device)), "df_train_apply")

    def step(self, xbuf, thbuf, batch: int, lpsum=None):
        _lib.check(self.lib.df_train_step(self.handle, _ptr(xbuf), _ptr(thbuf), C.c_int64(batch), _ptr(lpsum),
                                          _stream(self.device)), "df_train_step")

    def step_graph(self, xbuf, thbuf, batch: int, n_total: int = None, lpsum=None):
        """gradient + apply replayed as one hipGraph once the same buffers repeat
        (df_train_step_graph); pass persistent staging buffers."""
        n_total = batch if n_total is None else n_total
        _lib.check(self.lib.df_train_step_graph(self.handle, _ptr(xbuf), _ptr(thbuf), C.c_int64(batch),
                                                C.c_int64(n_total), _ptr(lpsum), _stream(self.device)),
                   "df_train_step_graph")

    def sweep(self) -> int:
        """The reverse-sweep form this trainer runs (df_train_sweep: SWEEP_* | SWEEP_SEPARATE)."""
        f = C.c_int()
        _lib.check(self.lib.df_train_sweep(self.handle, C.byref(f)), "df_train_sweep")
        return int(f.value)

    def set_debug(self, on: bool = True) -> None:
        """train!(...; debug=true): refuse the Adam update of a non-finite loss
        (df_train_set_debug → NonFiniteError)."""
        _lib.check(self.lib.df_train_set_debug(self.handle, 1 if on else 0))

    def set_theta_input(self, mode: int) -> None:
        """df_train_set_theta_input: _lib.DF_THETA_AUTO (default; normalise θ iff the
        chain has bounds), DF_THETA_RAW (always normalise) or DF_THETA_GIVEN (never)."""
        _lib.check(self.lib.df_train_set_theta_input(self.handle, int(mode)), "df_train_set_theta_input")

    def allreduce_gradient(self, comm) -> None:
        """Sum the flat gradient over the ranks of ``comm`` (df_train_allreduce_gradient)."""
        _lib.check(self.lib.df_train_allreduce_gradient(self.handle, comm.handle, _stream(self.device)),
                   "df_train_allreduce_gradient")

    def step_dist(self, comm, xbuf, thbuf, batch: int, n_total: int, lpsum=None):
        """One data-parallel step on this rank's shard (df_train_step_dist):
        gradient (mean over the global ``n_total``) → RCCL all-reduce → Adam."""
        _lib.check(self.lib.df_train_step_dist(self.handle, comm.handle if comm is not None else None, _ptr(xbuf),
                                               _ptr(thbuf), C.c_int64(batch), C.c_int64(n_total), _ptr(lpsum),
                                               _stream(self.device)), "df_train_step_dist")

    def get_params(self) -> np.ndarray:
        out = np.empty(self.num_params, dtype=np.float32)
        _lib.check(self.lib.df_train_get_params(self.handle, out.ctypes.data_as(C.POINTER(C.c_float)),
                                                C.c_int64(self.num_params)))
        return out

    def set_params(self, flat) -> None:
        flat = np.ascontiguousarray(flat, dtype=np.float32).reshape(-1)
        _lib.check(self.lib.df_train_set_params(self.handle, flat.ctypes.data_as(C.POINTER(C.c_float)),
                                                C.c_int64(flat.shape[0])))


def _dense_order(elements):
    """Dense layers in Flux.trainables order (s_net then t_net per coupling layer)."""
    out = []
    for _, l in flatten_elements(elements):
        if isinstance(l, NormalizationLayer):
            continue
        if isinstance(l, RNVPCouplingLayer):
            out += list(l.s_net)
        out += list(l.t_net)
    return out


def trainables(model) -> np.ndarray:
    """``Flux.trainables(model)`` flattened: per Dense vec(weight) then bias."""
    parts = []
    for D in _dense_order(model.layers):
        parts.append(np.asarray(D.W, np.float32).ravel(order="F"))
        if D.b is not None:
            parts.append(np.asarray(D.b, np.float32))
    return np.concatenate(parts) if parts else np.zeros(0, np.float32)


def load_trainables(model, flat) -> None:
    """Write a flat trainables vector back into the model's Dense layers."""
    flat = np.asarray(flat, np.float32)
    o = 0
    for D in _dense_order(model.layers):
        k = D.W.size
        D.W = flat[o:o + k].reshape(D.W.shape, order="F").copy()
        o += k
        if D.b is not None:
            D.b = flat[o:o + D.b.size].copy()
            o += D.b.size
    if o != flat.shape[0]:
        raise _lib.DimensionMismatch(f"trainables length {flat.shape[0]} does not match the model ({o})")


class TrainState:
    """``Optimisers.setup(opt, flow.model)``: the device-resident optimiser state."""

    def __init__(self, flow, opt: Adam, device=None):
        self.flow = flow
        self.opt = opt
        self.trainer = HIPTrainer(flow.hip(device), opt)

    def sync_model(self):
        """Copy the device parameters back into the Python model (Dense.W / .b)."""
        load_trainables(self.flow.model, self.trainer.get_params())


def setup(opt: Adam, flow, device=None) -> TrainState:
    return TrainState(flow, opt, device)


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def _loss(flow, x, th, group=None, comm=None):
    """loss(backward(model, x, θ)...) over a whole set (fused NLL, fp64 sum).
    With a ``DFComm`` the set is sharded over its ranks and reduced inside the
    library (df_flow_nll); under a bare torch.distributed group (the gloo
    rehearsal) the 16-byte partial goes through torch."""
    import torch

    from .parallel import allreduce_nll, flow_nll, shard_range

    B = x.shape[1]
    dist = _dist()
    if comm is not None:
        a, b = shard_range(B, comm.rank, comm.world)
        return flow_nll(flow, x[:, a:b], th[:, a:b] if th is not None else None, comm)[0]
    if dist is not None:
        r, w = dist.get_rank(group), dist.get_world_size(group)
        a, b = shard_range(B, r, w)
        x, th = x[:, a:b], (th[:, a:b] if th is not None else None)
    h = flow.hip()
    s = torch.zeros(1, dtype=torch.float64, device=h.device)
    if x.shape[1] > 0:
        h.logpdf_sum(x, th, out=s)
    loss, _, _ = allreduce_nll(s, x.shape[1], group)
    return loss


def _nonfinite(v: float) -> bool:
    return not np.isfinite(v)


def train_(flow, data, state: TrainState, epochs: int = 100, batchsize: int = 64, shuffle: bool = True,
           verbose: bool = True, debug: bool = False, rng=None, group=None, graphs: bool = True, comm=None):
    """``train!(flow, data, opt_state; epochs, batchsize, shuffle, verbose, debug)`` — src/Flows.jl:380-445.

    Per epoch: mini-batches of the training split (Flux.DataLoader: reshuffled
    every epoch when ``shuffle``, last partial batch kept), one gradient + Adam
    step each; then the train and validation losses are pushed to
    ``flow.train_loss`` / ``flow.valid_loss``.  θ is normalised with the
    Flow's MetaData inside the kernels (= normalized_training_data, Data.jl:189).

    ``debug`` (src/Flows.jl:404-409,423-435): a mini-batch whose loss is NaN
    or ±Inf raises ``ArgumentError`` before its update (the library refuses
    the Adam step, DF_ERR_NONFINITE); a non-finite epoch train / valid loss
    prints the reference's message and returns ``backward(model, set...)``
    = (z, ldj); a run that completes returns (None, None).

    Data parallelism: with ``comm`` (a :class:`DFComm`, one rank per GPU)
    every batch is sharded over its ranks and each step is
    ``df_train_step_dist`` (gradient over the global mean → RCCL all-reduce
    inside the library → Adam); the epoch losses use ``df_flow_nll``.  Under
    a torch.distributed group without ``comm`` (the CPU/gloo rehearsal) the
    gradient goes through torch's all-reduce.  Every rank must pass the same
    ``rng`` seed.  On one device each mini-batch is gathered into a
    persistent staging buffer and the step (reverse sweep, reduction, Adam,
    repack) is replayed as one hipGraph (``graphs``; df_train_step_graph),
    which removes the per-launch host overhead that dominates the reference's
    default batchsize of 64."""
    import torch

    from .parallel import shard_range

    rng = rng if rng is not None else np.random.default_rng()
    tr = state.trainer
    tr.set_debug(debug)
    dev = tr.device
    x_tr, th_tr = data.training_data()
    x_va, th_va = data.validation_data()
    n = flow.n
    xt, _, _ = as_julia_device(x_tr, flow.d, dev, "x")          # (N*d,) Julia order
    tt = as_julia_device(th_tr, n, dev, "θ")[0] if n > 0 else None
    N = x_tr.shape[1]
    Xs = xt.view(N, flow.d)                                      # row j = sample j
    Ts = tt.view(N, n) if tt is not None else None
    dist = _dist()
    if comm is not None:
        rank, world = comm.rank, comm.world
    else:
        rank, world = (dist.get_rank(group), dist.get_world_size(group)) if dist is not None else (0, 1)
    local = comm is None and dist is None
    staging = {}  # batch size → persistent (x, θ) device buffers (stable pointers for the graphs)
    for _ in range(epochs):
        order = rng.permutation(N) if shuffle else np.arange(N)
        for b0 in range(0, N, batchsize):
            idx = order[b0:b0 + batchsize]
            B = idx.shape[0]
            a, b = shard_range(B, rank, world)
            ii = torch.as_tensor(idx[a:b], device=dev)
            try:
                if local and graphs:
                    if B not in staging:
                        staging[B] = (torch.empty((B, flow.d), dtype=Xs.dtype, device=dev),
                                      torch.empty((B, n), dtype=Ts.dtype, device=dev) if Ts is not None else None)
                    xb, tb = staging[B]
                    torch.index_select(Xs, 0, ii, out=xb)
                    if Ts is not None:
                        torch.index_select(Ts, 0, ii, out=tb)
                    tr.step_graph(xb, tb, B)
                    continue
                xb = Xs.index_select(0, ii).contiguous()
                tb = Ts.index_select(0, ii).contiguous() if Ts is not None else None
                if local:
                    tr.step(xb, tb, B)
                elif comm is not None:
                    tr.step_dist(comm, xb, tb, b - a, B)
                else:
                    tr.gradient(xb, tb, b - a, B)
                    dist.all_reduce(tr.grad(), op=dist.ReduceOp.SUM, group=group)
                    if debug:  # the rehearsal's loss check: global Σ logpdf through torch
                        lp = torch.zeros(1, dtype=torch.float64, device=dev)
                        if b > a:
                            flow.hip().logpdf_sum(xb.T, tb.T if tb is not None else None, out=lp)
                        dist.all_reduce(lp, op=dist.ReduceOp.SUM, group=group)
                        if _nonfinite(float(lp.item())):
                            raise _lib.NonFiniteError(f"non-finite training loss {-float(lp.item()) / B}")
                    tr.apply()
            except _lib.NonFiniteError as e:
                # the reference throws from inside the gradient closure, after printing
                # "$l, $ln_det_jac, $z" of the batch (src/Flows.jl:404-409); update! has
                # left flow.model at the last good parameters, and so does sync_model here
                state.sync_model()
                if rank == 0:
                    xv = xb[: b - a].T if local and graphs else xb.T
                    tv = (tb[: b - a].T if local and graphs else tb.T) if tb is not None else None
                    z, ldj = flow.backward(xv, tv)
                    s = flow.hip().logpdf_sum(xv, tv)[0]
                    print(f"{-float(s.item()) / max(b - a, 1)}, {ldj.cpu().numpy()}, {z.cpu().numpy()}")
                raise _lib.ArgumentError(str(e)) from e
        train_loss = _loss(flow, x_tr, th_tr if n > 0 else None, group, comm)
        flow.train_loss.append(train_loss)
        if debug and _nonfinite(train_loss):
            if rank == 0:
                print(f"Problem with train loss {train_loss}")
            state.sync_model()
            return _backward_set(flow, x_tr, th_tr)
        valid_loss = _loss(flow, x_va, th_va if n > 0 else None, group, comm)
        flow.valid_loss.append(valid_loss)
        if debug and _nonfinite(valid_loss):
            if rank == 0:
                print(f"Problem with valid loss {valid_loss}")
            state.sync_model()
            return _backward_set(flow, x_va, th_va)
        if verbose and rank == 0:
            print(f"epoch: {len(flow.train_loss)} | train_loss = {train_loss}, valid_loss = {valid_loss}")
    state.sync_model()
    return (None, None) if debug else None


def _backward_set(flow, x, th):
    """``backward(flow.model, set...)`` on a normalised data set: (z, ldj)."""
    return flow.backward(x, th if flow.n > 0 else None)
