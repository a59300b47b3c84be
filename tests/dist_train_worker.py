"""Worker of tests/test_gpu_train.py::test_data_parallel_train_matches_single:
one rank of a data-parallel train! run (launched by torch.distributed.run)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]


def build(rng_seed=0):
    import densityflows_amd as dfa

    x = np.load(os.path.join(HERE, "golden", "datatest_x.npy"))
    th = np.load(os.path.join(HERE, "golden", "datatest_theta.npy"))
    rng = np.random.default_rng(rng_seed)
    data = dfa.DataArrays(x, th, rng=rng)
    chain = dfa.FlowChain(
        dfa.CouplingLayer(data, [1, 2, 3], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.CouplingLayer(data, [3, 4, 5], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.CouplingLayer(data, [5, 1, 2], hidden_dim_s=16, hidden_dim_t=16, rng=rng),
        dfa.NormalizationLayer.from_data(x, -1.0, 1.0))
    return data, chain, dfa.Flow(chain, data)


def run(group=None, epochs=2, comm=None, graphs=True):
    import densityflows_amd as dfa
    from densityflows_amd.train import trainables

    data, chain, flow = build()
    state = dfa.setup(dfa.Adam(1e-3), flow)
    dfa.train_(flow, data, state, epochs=epochs, batchsize=64, verbose=False, rng=np.random.default_rng(1),
               group=group, comm=comm, graphs=graphs)
    return trainables(chain), np.asarray(flow.train_loss), np.asarray(flow.valid_loss)


if __name__ == "__main__":
    import torch
    import torch.distributed as dist

    rccl = len(sys.argv) > 2 and sys.argv[2] == "rccl"
    rank = int(os.environ["RANK"])
    comm = None
    # gloo carries the bootstrap (and, in the rehearsal, the gradient); with "rccl" every
    # rank owns its GPU and the library's communicator carries every exchange
    torch.cuda.set_device(rank if rccl else 0)
    dist.init_process_group("gloo")
    if rccl:
        from densityflows_amd.parallel import DFComm

        comm = DFComm(rank, rank, dist.get_world_size())
    p, tl, vl = run(comm=comm)
    if comm is not None:
        comm.close()
    if dist.get_rank() == 0:
        np.savez(sys.argv[1], params=p, train_loss=tl, valid_loss=vl)
    dist.barrier()
    dist.destroy_process_group()
