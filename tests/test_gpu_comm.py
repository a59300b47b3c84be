"""Multi-GPU exchange on the GPU: the library's RCCL communicator (df_comm_*)
and the sharded NLL of config 3 (src/Flows.jl:352-359), plus the
data-parallel train! step (df_train_step_dist, src/Flows.jl:398-413).

On a one-GPU box the RCCL path runs as a world-1 communicator (the real
ncclCommInitRank / ncclAllReduce calls); the 2-rank case is rehearsed with
gloo carrying the same 16-byte {Σ, count}."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import densityflows_amd as dfa
import make_golden as G
from helpers import spec_to_element

pytestmark = pytest.mark.gpu


def _t(a, dev):
    import torch

    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float32).T)).to(dev).T


@pytest.fixture(scope="module")
def comm(cuda):
    from densityflows_amd.parallel import DFComm

    c = DFComm(0)
    yield c
    c.close()


def test_world1_comm_info_and_allreduce(cuda, comm):
    import torch

    assert comm.info() == (0, 1, 0)
    a = torch.arange(1000, dtype=torch.float32, device=cuda)
    ref = a.clone()
    comm.allreduce_(a)
    d = torch.linspace(-1, 1, 17, dtype=torch.float64, device=cuda)
    dref = d.clone()
    comm.allreduce_(d)
    torch.cuda.synchronize()
    assert torch.equal(a, ref) and torch.equal(d, dref)


@pytest.mark.parametrize("name", ["cfg2", "cfg1"])
def test_world1_rccl_nll_matches_golden(cuda, comm, name):
    """df_flow_nll through a real RCCL communicator: {Σ, N} all-reduced, loss =
    -mean(golden logpdf); Σ is bitwise the local df_flow_logpdf_sum."""
    from densityflows_amd.parallel import flow_nll

    spec, g, meta = G.load(name)
    flow = dfa.Flow(spec_to_element(spec), metadata=dfa.MetaData("", meta["d"], meta["n"], g["theta_min"],
                                                                 g["theta_max"]))
    th = _t(g["theta_raw"], cuda) if meta["n"] > 0 else None
    loss, s, n = flow_nll(flow, _t(g["x_in"], cuda), th, comm)
    assert n == meta["B"]
    ref = -float(np.mean(g["logpdf"].astype(np.float64)))
    assert abs(loss - ref) <= 1e-5 * abs(ref), (loss, ref)
    s_local, _ = dfa.nll_partial_sum(flow, _t(g["x_in"], cuda), th)
    assert float(s_local.item()) == s


def test_world1_train_step_dist_equals_local_step(cuda, comm):
    """df_train_step_dist with a world-1 communicator (gradient → ncclAllReduce →
    Adam) is bitwise the plain df_train_step."""
    import torch

    from densityflows_amd.train import Adam, HIPTrainer

    spec, g, meta = G.load("cfg1")
    B = 2048
    x = torch.from_numpy(np.ascontiguousarray(g["x_in"][:, :B].T)).to(cuda).reshape(-1)
    th = torch.from_numpy(np.ascontiguousarray(g["theta_raw"][:, :B].T)).to(cuda).reshape(-1)
    out = []
    for dist_step in (False, True):
        flow = dfa.Flow(spec_to_element(spec), metadata=dfa.MetaData("", meta["d"], meta["n"], g["theta_min"],
                                                                     g["theta_max"]))
        tr = HIPTrainer(flow.hip(), Adam(1e-3))
        lp = torch.zeros(1, dtype=torch.float64, device=cuda)
        for _ in range(3):
            if dist_step:
                tr.step_dist(comm, x, th, B, B, lp)
            else:
                tr.step(x, th, B, lp)
        torch.cuda.synchronize()
        out.append((tr.get_params(), float(lp.item())))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_two_rank_sharded_nll_gloo(cuda, tmp_path):
    """Config-3 rehearsal: 2 ranks shard the cfg2 golden x_in; the reduced
    {Σ, N} of their df_flow_nll partials gives -mean(golden logpdf)."""
    _, g, meta = G.load("cfg2")
    out = str(tmp_path / "nll.npz")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(os.path.dirname(__file__), "dist_nll_worker.py"), out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = np.load(out)
    assert res["count"] == meta["B"] and res["shard_count"] == meta["B"] // 2
    ref = -float(np.mean(g["logpdf"].astype(np.float64)))
    loss = -float(res["sum"]) / float(res["count"])
    assert abs(loss - ref) <= 1e-5 * abs(ref), (loss, ref)
    # the shard partial is the fp64 sum of the golden logpdf over rank 0's half
    half = g["logpdf"][: meta["B"] // 2].astype(np.float64)
    assert abs(float(res["shard_sum"]) - half.sum()) <= 1e-5 * np.abs(half).sum()


def test_world1_train_with_comm_matches_local(cuda, comm):
    """train_(..., comm=DFComm) — df_train_step_dist per mini-batch, df_flow_nll per
    epoch — through a real world-1 RCCL communicator equals the local train_ bitwise:
    parameters and the train / valid loss vectors (src/Flows.jl:380-445)."""
    import dist_train_worker as W

    local = W.run(graphs=False)
    dist = W.run(comm=comm)
    np.testing.assert_array_equal(local[0], dist[0])
    np.testing.assert_array_equal(local[1], dist[1])
    np.testing.assert_array_equal(local[2], dist[2])


def test_two_rank_rccl_train(cuda, tmp_path):
    """Two ranks, one GPU each, the library's RCCL communicator for every exchange
    (gradient all-reduce, {Σ, N} of the epoch losses): the data-parallel train_ matches
    one process on the same batches to the gradient tolerance (the shard sums
    reassociate the batch mean).  Needs two GPUs."""
    import torch

    import dist_train_worker as W

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (one rank per GPU)")
    out = str(tmp_path / "rccl_train.npz")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(os.path.dirname(__file__), "dist_train_worker.py"), out, "rccl"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = np.load(out)
    p1, tl1, vl1 = W.run()
    np.testing.assert_allclose(res["train_loss"], tl1, rtol=1e-4)
    np.testing.assert_allclose(res["valid_loss"], vl1, rtol=1e-4)
    # as the gloo rehearsal (test_gpu_train.py): Adam normalises each step to ≈ η, so
    # reassociated gradient sums move near-zero-gradient coordinates by O(η)
    assert np.max(np.abs(res["params"] - p1)) <= 2e-3
    assert np.mean(np.abs(res["params"] - p1)) <= 2e-5
