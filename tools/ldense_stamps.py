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
       python tools/ldense_stamps.py --ldw [batch]   (the split dW1 kernel, tools/ldw_stamps_patch.py)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ldw_report(st):
    """tools/ldw_stamps_patch.py stamps: per wave, cycles of each step's phases."""
    for wg in range(2):
        t0 = st[wg, :, 0].min()
        print(f"workgroup {128 * wg}: per step (wait+barrier / split / barrier / MFMA issue), cycles")
        for w in range(4):
            row = st[wg, w]
            parts = []
            for k in range(31):
                ev = row[1 + 4 * k:5 + 4 * k + 1] - t0
                if row[1 + 4 * k] == 0 or row[5 + 4 * k] == 0:
                    break
                prev = row[4 * k] - t0 if k else 0
                parts.append(f"{ev[0] - prev}/{ev[1] - ev[0]}/{ev[2] - ev[1]}/{ev[3] - ev[2]}")
            print(f"  w{w} end {row[127] - t0}: " + " ".join(parts))


def main():
    import torch

    import bench
    from densityflows_amd.train import Adam, HIPTrainer

    args = [a for a in sys.argv[1:] if a != "--ldw"]
    B = int(args[0]) if args else 1 << 18
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
        if LDW:
            wb = np.zeros(2 * 4 * 128, np.uint64)
            assert lib.df_diag_ldw_stamps(wb.ctypes.data_as(ctypes.c_void_p)) == 0
            print(f"rep {rep}")
            ldw_report(wb.reshape(2, 4, 128).astype(np.int64))
            continue
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


LDW = "--ldw" in sys.argv

if __name__ == "__main__":
    main()
