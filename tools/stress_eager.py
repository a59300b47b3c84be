"""GPU box: hunt the rare eager-step non-reproducibility of test_step_graph_matches_eager_steps
(DESIGN §7).  The test's E (eager) / G (graph) sequence is repeated after "poisoning" the
device allocator: a large trainer is stepped and destroyed first, so the buffers the next
trainers allocate at their capacity growth (step 8, B = 5000) come back holding old data
instead of fresh zero pages.  Each rep also replays the sequence on a third eager trainer R
and reports the first step at which E, G and R disagree.
    python tools/stress_eager.py <readme|cfg2|mixed|cfg5> [reps] [sweep]"""
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sweep = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    cuda = torch.device("cuda", 0)
    seq = (64, 64, 64, 64, 33, 33, 33, 64, 5000, 5000, 5000, 64, 64)
    spec, _, d, n = T._setup(name, seed=7)

    def poison(rep):
        # a trainer with a large capacity whose buffers hold data, then freed
        big = HIPTrainer(spec_to_element(spec).hip(device=0), Adam(1e-3), sweep=sweep)
        x, th = T._inputs(d, n, 40000 + 1000 * rep, seed=100 + rep)
        big.step(T._dev(x, cuda), T._dev(th, cuda) if n else None, x.shape[1])
        torch.cuda.synchronize()
        del big

    def run(trainers, graph_idx=None):
        hist = [[] for _ in trainers]
        bufs = {}
        for B in seq:
            x, th = T._inputs(d, n, B, seed=B)
            xd, td = T._dev(x, cuda), (T._dev(th, cuda) if n else None)
            if B not in bufs:
                bufs[B] = (torch.empty_like(xd), torch.empty_like(td) if n else None)
            xs, ts = bufs[B]
            xs.copy_(xd)
            if n:
                ts.copy_(td)
            for k, tr in enumerate(trainers):
                if k == graph_idx:
                    tr.step_graph(xs, ts, B)
                else:
                    tr.step(xd, td, B)
            torch.cuda.synchronize()
            for k, tr in enumerate(trainers):
                hist[k].append(tr.get_params().copy())
        return hist

    bad = 0
    for rep in range(reps):
        poison(rep)
        E = HIPTrainer(spec_to_element(spec).hip(device=0), Adam(1e-3), sweep=sweep)
        G = HIPTrainer(spec_to_element(spec).hip(device=0), Adam(1e-3), sweep=sweep)
        he, hg = run([E, G], graph_idx=1)
        del E, G
        poison(rep + 7)
        R = HIPTrainer(spec_to_element(spec).hip(device=0), Adam(1e-3), sweep=sweep)
        (hr,) = run([R])
        del R
        first = {}
        for a_name, ha in (("E", he), ("G", hg)):
            for i in range(len(seq)):
                if not np.array_equal(ha[i], hr[i]):
                    first[a_name] = i
                    break
        if first:
            bad += 1
        print(f"{name} sweep {sweep} rep {rep}: first step differing from the replay R: {first or 'none'}",
              flush=True)
    print(f"{name} sweep {sweep}: {bad} of {reps} reps disagree", flush=True)


if __name__ == "__main__":
    main()
