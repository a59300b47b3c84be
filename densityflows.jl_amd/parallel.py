"""Multi-GPU data parallelism over samples (one process per GPU).

The FlowChain forward / inverse passes are independent per sample
(src/Chains.jl:149-197): every rank evaluates its own contiguous block of the
batch with its own device handle and nothing is exchanged.  The only
cross-sample quantity is the NLL ``loss = -mean(logpdf)`` (src/Flows.jl:352-359):
each rank produces an fp64 partial Σ logpdf on device (``df_flow_logpdf_sum``)
and a single all-reduce of ``{Σ, count}`` (16 bytes; RCCL over xGMI with the
``nccl`` backend, gloo on CPU) gives the global mean.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

from . import _lib

__all__ = ["shard_range", "allreduce_nll", "distributed_nll", "DFComm", "flow_nll"]


def shard_range(batch: int, rank: int, world: int) -> Tuple[int, int]:
    """[start, stop) of rank's contiguous block; sizes differ by at most one sample."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("invalid rank / world size")
    base, extra = divmod(int(batch), world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def allreduce_nll(partial_sum, count, group=None):
    """All-reduce {Σ logpdf, count} and return (loss, Σ, total count) as floats.

    ``partial_sum`` is a 1-element float64 tensor on this rank's device (or CPU
    for gloo); ``count`` the number of samples it covers."""
    import torch
    import torch.distributed as dist

    buf = torch.zeros(2, dtype=torch.float64, device=partial_sum.device)
    buf[0] = partial_sum.reshape(-1)[0]
    buf[1] = float(count)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    total, n = float(buf[0].item()), float(buf[1].item())
    return (-total / n if n > 0 else float("nan")), total, n


def distributed_nll(flow, x_shard, theta_shard=None, group=None):
    """NLL of the full batch from per-rank shards (fused inverse + logpdf + Σ)."""
    from .flows import nll_partial_sum

    s, cnt = nll_partial_sum(flow, x_shard, theta_shard)
    return allreduce_nll(s, cnt, group)


class DFComm:
    """A ``df_comm`` handle: the library's own RCCL communicator (one rank per
    GPU, xGMI).  Every cross-rank exchange of the hot path goes through it —
    the NLL ``{Σ logpdf, count}`` (``df_flow_nll``) and the flat gradient
    (``df_train_allreduce_gradient`` / ``df_train_step_dist``).

    The 128-byte RCCL unique id is created on rank 0 and shipped to the other
    ranks over an already initialised ``torch.distributed`` group (any
    backend) — the out-of-band bootstrap a Julia host would do with MPI or a
    file.  ``world == 1`` needs no process group."""

    def __init__(self, device: int, rank: int = 0, world: int = 1, group=None, uid: Optional[bytes] = None):
        self.lib = _lib.load()
        if uid is None:
            uid = self.unique_id() if rank == 0 else None
            if world > 1:
                import torch.distributed as dist

                box = [uid]
                dist.broadcast_object_list(box, src=0, group=group)
                uid = box[0]
        if uid is None or len(uid) != _lib.DF_COMM_ID_BYTES:
            raise _lib.ArgumentError("invalid RCCL unique id")
        self._uid = C.create_string_buffer(bytes(uid), _lib.DF_COMM_ID_BYTES)
        h = C.c_void_p()
        _lib.check(self.lib.df_comm_init_rank(C.byref(h), int(world), self._uid, int(rank), int(device)),
                   "df_comm_init_rank")
        self.handle = h
        self.rank, self.world, self.device_index = int(rank), int(world), int(device)

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(_lib.DF_COMM_ID_BYTES)
        _lib.check(_lib.load().df_comm_get_unique_id(buf), "df_comm_get_unique_id")
        return buf.raw

    @classmethod
    def from_torch(cls, device: int, group=None) -> "DFComm":
        """Rank / world size from the initialised torch.distributed group (or 1 rank)."""
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return cls(device, dist.get_rank(group), dist.get_world_size(group), group)
        return cls(device)

    def info(self):
        r, w, d = C.c_int(), C.c_int(), C.c_int()
        _lib.check(self.lib.df_comm_get_info(self.handle, C.byref(r), C.byref(w), C.byref(d)))
        return r.value, w.value, d.value

    def allreduce_(self, t):
        """In-place sum over the ranks of a float32 / float64 device tensor (stream-ordered)."""
        import torch

        dt = {torch.float32: _lib.DF_DTYPE_F32, torch.float64: _lib.DF_DTYPE_F64}.get(t.dtype)
        if dt is None or not t.is_contiguous() or t.device.type != "cuda":
            raise _lib.ArgumentError("allreduce_ needs a contiguous float32/float64 device tensor")
        stream = C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
        _lib.check(self.lib.df_comm_allreduce_sum(self.handle, C.c_void_p(t.data_ptr()), C.c_int64(t.numel()), dt,
                                                  stream), "df_comm_allreduce_sum")
        return t

    def close(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self.handle = None
            _lib.check(self.lib.df_comm_destroy(h), "df_comm_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


def flow_nll(flow, x_shard, theta_shard=None, comm: Optional[DFComm] = None, out=None):
    """``loss`` (src/Flows.jl:352-359) of a sharded batch through ``df_flow_nll``:
    fused inverse + logpdf + fp64 Σ of this rank's shard, then the RCCL
    all-reduce of ``{Σ, count}`` inside the library.  Returns (loss, Σ, N)."""
    import torch

    from .hip import _ptr, _stream

    h = flow.hip()
    th = flow._theta(theta_shard, x_shard)
    xb, thb, dims, batch, _ = h._inputs(x_shard, th, "x")
    s = out if out is not None else torch.empty(2, dtype=torch.float64, device=h.device)
    _lib.check(h.lib.df_flow_nll(h.handle, comm.handle if comm is not None else None, _ptr(xb), _ptr(thb),
                                 C.c_int64(batch), C.c_void_p(s.data_ptr()), _stream(h.device)), "df_flow_nll")
    total, n = float(s[0].item()), float(s[1].item())
    return (-total / n if n > 0 else float("nan")), total, n
