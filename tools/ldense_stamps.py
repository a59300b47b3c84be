"""Phase timeline of the config-5 W1ᵀδ1 kernel (ldense_kernel<16,0,5,SPLIT>), diagnostic.

Needs a library built from the instrumented source (tools/ldense_stamps_patch.py, then
OBJS=df_ltrain tools/build_variant.sh lst "-DDF_LDENSE_STAMPS"), selected with
DENSITYFLOWS_HIP_LIB.  Every wave of workgroups 0 and 128 (the patch's second workgroup)
stores s_memtime (shader cycles) at: 0 start of the round loop; per round r (base 1 + 24r):
+0 round start, +1 + c after chunk c's wait and barrier, +9 epilogue start, +10 round end,
and per tile t of the epilogue +11 + 4t tile start, +12 + 4t δ0 stored, +13 + 4t x̄ product
issued, +14 + 4t z̄ stored; 120 after the final drain.  The last launch of a config-5
gradient (net 0's W1ᵀδ1) is the one read back.
usage: python tools/ldense_stamps.py [batch]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from densityflows_amd.train import Adam, HIPTrainer

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    dev = torch.device("cuda", 0)
    d, n, _ = bench.CONFIGS["cfg4"]
    chain = bench.build_chain("cfg4")
    hc = chain.hip(device=0, n_hint=n)
    hc.set_theta_bounds(np.zeros(n, np.float32), np.ones(n, np.float32))
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(B * d, device=dev, generator=g)
    th = torch.rand(B * n, device=dev, generator=g)
    tr = HIPTrainer(hc, Adam(1e-3))
    lib = ctypes.CDLL(os.environ["DENSITYFLOWS_HIP_LIB"])
    buf = np.zeros(2 * 8 * 128, np.uint64)
    for rep in range(3):
        tr.gradient(x, th, B, B)
        torch.cuda.synchronize()
        rc = lib.df_diag_ldense_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0, rc
        st = buf.reshape(2, 8, 128).astype(np.int64)
        for wg in range(2):
            t0 = st[wg, :, 0].min()
            print(f"rep {rep} workgroup {128 * wg}: cycles from the first wave's loop start")
            for w in range(8):
                row = st[wg, w]
                out = [f"w{w} end {row[120] - t0:7d}"]
                for r in range(4):
                    b = 1 + 24 * r
                    ev = row[b:b + 19] - t0
                    if row[b] == 0:
                        break
                    ch = np.diff(ev[1:10])
                    out.append(f"r{r} start {ev[0]:7d} c0 +{ev[1] - ev[0]:5d} chunks {' '.join(str(v) for v in ch)}"
                               f" epi {ev[10] - ev[9]:5d} [" + " ".join(
                                   f"t{t}: {ev[11 + 4 * t] - ev[9]} δ0 +{ev[12 + 4 * t] - ev[11 + 4 * t]}"
                                   f" x̄ +{ev[13 + 4 * t] - ev[12 + 4 * t]} z̄ +{ev[14 + 4 * t] - ev[13 + 4 * t]}"
                                   for t in range(2)) + "]")
                print("  " + "\n    ".join(out))


if __name__ == "__main__":
    main()
