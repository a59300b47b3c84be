"""Phase timeline of workgroup 0 / wave 0 of the specialised chain kernel (diagnostic).

Needs a library built with -DDF_PHASE_STAMPS (tools/build_variant.sh ph "-DDF_PHASE_STAMPS"),
selected with DENSITYFLOWS_HIP_LIB: the kernel then writes, into x[1..10] of the forward
output, the shader-cycle offsets (s_memtime) of its phases from the wave's start:
  1 table copy, 2 z copy-in, 3 θ copy-in + state init, 4 barrier, 5-8 after layers 0-3,
  9 copy-out issued, 10 copy-out drained, 11 layer 1 before its s-net, 12 after it.
usage: python tools/phase_stamps.py [config] [batch] [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench

    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg1"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    d, n, _ = bench.CONFIGS[cfg]
    chain = bench.build_chain(cfg)
    hc = chain.hip(device=0, n_hint=n)
    dev = torch.device("cuda", 0)
    z = torch.randn(B * d, device=dev)
    th = torch.rand(B * n, device=dev) if n else None
    x = torch.empty_like(z)
    ldj = torch.empty(B, device=dev)
    rows = []
    for r in range(reps):
        hc.run("forward", z, th, x, ldj, B)
        if r >= reps - 20:
            torch.cuda.synchronize()
            rows.append(x[1:14].cpu().numpy().astype(np.int64))
    rows = np.array(rows)
    med = np.median(rows, axis=0)
    names = ["tables", "z in", "theta in+init", "barrier", "layer0", "layer1", "layer2", "layer3",
             "copy-out issued", "copy-out drained", "L1 kind read", "L1 s-net", "L1 descr. loaded"]
    prev = 0
    print(f"{cfg} B={B}: cycles from wave start (median of 20 launches), and the phase's own share")
    for nm, v in zip(names, med):
        print(f"  {nm:18s} {v:9.0f}  (+{v - prev:.0f})")
        prev = v


if __name__ == "__main__":
    main()
