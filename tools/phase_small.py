"""Phase timeline of workgroup 0 of the small-batch kernel (diagnostic; df_small.hip built
with -DDF_PHASE_STAMPS, selected with DENSITYFLOWS_HIP_LIB): x[1..7] of the forward output
hold the s_memtime offsets of 1 loads + LDS row, 2-5 after layers 0-3, 6 stores issued,
7 stores drained.  usage: python tools/phase_small.py [batch]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    chain = bench.build_chain("cfg1")
    hc = chain.hip(device=0, n_hint=1)
    dev = torch.device("cuda", 0)
    z = torch.randn(B * 5, device=dev)
    th = torch.rand(B, device=dev)
    x = torch.empty_like(z)
    ldj = torch.empty(B, device=dev)
    rows = []
    for r in range(200):
        hc.run("forward", z, th, x, ldj, B)
        if r >= 180:
            torch.cuda.synchronize()
            rows.append(x[1:8].cpu().numpy().astype(np.int64))
    med = np.median(np.array(rows), axis=0)
    prev = 0
    for nm, v in zip(["loads+row", "layer0", "layer1", "layer2", "layer3(norm)", "stores issued", "drained"], med):
        print(f"  {nm:14s} {v:8.0f} (+{v - prev:.0f})")
        prev = v


if __name__ == "__main__":
    main()
