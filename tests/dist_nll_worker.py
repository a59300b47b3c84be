"""Worker of tests/test_gpu_comm.py::test_two_rank_sharded_nll_gloo: one rank
of the config-3 sharded NLL (src/Flows.jl:352-359) rehearsed on one GPU.

Each rank takes its contiguous shard of the config-2 golden x_in, runs
df_flow_nll with no communicator (this rank's fused inverse + logpdf + fp64
Σ and its count), and the 16-byte {Σ, N} goes through a gloo all-reduce — the
exchange df_comm performs over RCCL when every rank owns a GPU (two ranks
cannot share one GPU in an RCCL communicator)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE, os.path.join(HERE, "golden")]


def main(out):
    import torch
    import torch.distributed as dist

    import densityflows_amd as dfa
    import make_golden as G
    from densityflows_amd.parallel import flow_nll, shard_range
    from helpers import spec_to_element

    torch.cuda.set_device(0)  # rehearsal: every rank shares GPU 0
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    spec, g, meta = G.load("cfg2")
    flow = dfa.Flow(spec_to_element(spec), metadata=dfa.MetaData("", meta["d"], meta["n"], g["theta_min"],
                                                                 g["theta_max"]))
    x = g["x_in"]
    a, b = shard_range(x.shape[1], rank, world)
    xs = torch.from_numpy(np.ascontiguousarray(x[:, a:b].T)).cuda().T
    _, s_local, n_local = flow_nll(flow, xs)                     # df_flow_nll, comm = NULL
    buf = torch.tensor([s_local, n_local], dtype=torch.float64)
    dist.all_reduce(buf)
    if rank == 0:
        np.savez(out, sum=buf[0].item(), count=buf[1].item(), shard_sum=s_local, shard_count=n_local)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
