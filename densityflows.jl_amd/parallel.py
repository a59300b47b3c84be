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

from typing import Tuple

__all__ = ["shard_range", "allreduce_nll", "distributed_nll"]


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
