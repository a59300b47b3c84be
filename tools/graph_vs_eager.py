"""GPU box: the sequence of test_step_graph_matches_eager_steps on one chain, repeated,
reporting at which step (if any) the graph-replayed trainer's parameters first differ
from the eager trainer's.  Layer-wise path requested by DENSITYFLOWS_SWEEP (a
df_sweep_form number; 0 = automatic).
    python tools/graph_vs_eager.py <readme|cfg2|mixed|cfg5> [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    import torch

    import test_gpu_train as T
    from densityflows_amd.train import Adam, HIPTrainer
    from helpers import spec_to_element

    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sweep = int(os.environ.get("DENSITYFLOWS_SWEEP", "0"))
    cuda = torch.device("cuda", 0)
    for rep in range(reps):
        spec, chain, d, n = T._setup(name, seed=7)
        chain2 = spec_to_element(spec)
        eager = HIPTrainer(chain.hip(device=0), Adam(1e-3), sweep=sweep)
        graph = HIPTrainer(chain2.hip(device=0), Adam(1e-3), sweep=sweep)
        bufs = {}
        first_bad = None
        for i, B in enumerate((64, 64, 64, 64, 33, 33, 33, 64, 5000, 5000, 5000, 64, 64)):
            x, th = T._inputs(d, n, B, seed=B)
            xd, td = T._dev(x, cuda), (T._dev(th, cuda) if n else None)
            if B not in bufs:
                bufs[B] = (torch.empty_like(xd), torch.empty_like(td) if n else None)
            xs, ts = bufs[B]
            xs.copy_(xd)
            if n:
                ts.copy_(td)
            eager.step(xd, td, B)
            graph.step_graph(xs, ts, B)
            torch.cuda.synchronize()
            if first_bad is None and not np.array_equal(graph.get_params(), eager.get_params()):
                first_bad = (i, B)
        try:
            form = eager.sweep()
        except AttributeError:  # a saved pre-ABI-5 library (DF_TRAIN_LAYERWISE=1 selects its path)
            form = "?"
        print(f"{name} sweep {sweep} rep {rep}: form {form} first mismatch {first_bad}", flush=True)


if __name__ == "__main__":
    main()
