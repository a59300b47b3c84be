"""Dump the chain-pass outputs of one library build (DENSITYFLOWS_HIP_LIB) on fixed
seeded inputs, for bitwise A/B comparisons between builds:
    python tools/dump_outputs.py out.npz         # one build
    python tools/dump_outputs.py --compare a.npz b.npz
Workloads: the bench's config-2 and config-4 models (forward, inverse, logpdf) and a
training gradient of each (config 4's is the config-5 sweep)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(path):
    import torch

    import bench
    from densityflows_amd.train import Adam, HIPTrainer

    dev = torch.device("cuda", 0)
    out = {}
    for cfg, B in (("cfg2", 1 << 16), ("cfg4", 1 << 12)):
        d, n, _ = bench.CONFIGS[cfg]
        chain = bench.build_chain(cfg)
        hc = chain.hip(device=0, n_hint=n)
        if n:
            hc.set_theta_bounds(np.zeros(n, np.float32), np.ones(n, np.float32))
        g = torch.Generator(device=dev).manual_seed(7)
        z = torch.randn(B * d, device=dev, generator=g)
        th = torch.rand(B * n, device=dev, generator=g) if n else None
        x, ldj = torch.empty_like(z), torch.empty(B, device=dev)
        hc.run("forward", z, th, x, ldj, B)
        zb, ldjb = torch.empty_like(z), torch.empty(B, device=dev)
        hc.run("backward", x, th, zb, ldjb, B)
        lp = torch.empty(B, device=dev)
        hc.run_logpdf(x, th, lp, B)
        for k, v in (("x", x), ("ldj", ldj), ("zb", zb), ("ldjb", ldjb), ("lp", lp)):
            out[f"{cfg}_{k}"] = v.cpu().numpy()
        tr = HIPTrainer(hc, Adam(1e-3))  # cfg4: the config-5 sweep (wide inverse pass)
        tr.gradient(x, th, B, B)
        torch.cuda.synchronize()
        out[f"{cfg}_grad"] = tr.grad().cpu().numpy()
        del tr
    np.savez(path, **out)
    print("dumped", path, {k: v.shape for k, v in out.items()})


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    same = True
    for k in sorted(A.files):
        eq = np.array_equal(A[k].view(np.uint32), Bz[k].view(np.uint32))
        diff = np.max(np.abs(A[k].astype(np.float64) - Bz[k])) if not eq else 0.0
        print(f"{k:12s} {'bitwise-identical' if eq else 'DIFFERS max|Δ| %.3g' % diff}")
        same &= eq
    print("ALL BITWISE IDENTICAL" if same else "DIFFERENT")
    return same


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    dump(sys.argv[1])
