"""Multi-process (world_size 2, gloo on CPU) coverage of the sharded NLL path:
shard_range covers the batch exactly once and allreduce_nll combines the
per-rank fp64 partials into the full-batch loss (src/Flows.jl:352-359).  The
per-rank partials here come from the CPU oracle (the GPU path produces them
with df_flow_logpdf_sum; tests/test_gpu_parity.py checks that against the
oracle)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from densityflows_amd.parallel import shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("B,world", [(10, 2), (11, 2), (1, 3), (0, 2), (1 << 20, 8), (1000003, 7)])
def test_shard_range_partitions(B, world):
    seen = 0
    prev = 0
    for r in range(world):
        a, b = shard_range(B, r, world)
        assert a == prev and b >= a
        seen += b - a
        prev = b
    assert seen == B and prev == B


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import make_golden as G
    from oracle import flow_oracle as O
    from densityflows_amd.parallel import allreduce_nll, shard_range

    spec, g, meta = G.load("cfg1")
    B = 1001
    a, b = shard_range(B, rank, world)
    lp = O.flow_logpdf(spec, g["x_in"][:, a:b], g["theta"][:, a:b], np.float64)
    part = torch.tensor([float(np.sum(lp))], dtype=torch.float64)
    loss, total, n = allreduce_nll(part, b - a)
    q.put((rank, loss, total, n))
    dist.destroy_process_group()


def test_allreduce_nll_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import make_golden as G
    from oracle import flow_oracle as O

    spec, g, _ = G.load("cfg1")
    lp = O.flow_logpdf(spec, g["x_in"][:, :1001], g["theta"][:, :1001], np.float64)
    want = -float(np.mean(lp))
    for rank, loss, total, n in res:
        assert n == 1001
        assert loss == pytest.approx(want, rel=1e-12)
