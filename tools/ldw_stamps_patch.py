"""Instrument df_ltrain.hip in place with phase stamps of the split dW1 kernel
(ldw_split_kernel, config-5 H0-free sweep; diagnostic only, the product source carries none):
    python tools/ldw_stamps_patch.py densityflows.jl_amd/csrc/df_ltrain.hip
    OBJS=df_ltrain bash tools/build_variant.sh lws "-DDF_LDW_STAMPS"
    git checkout densityflows.jl_amd/csrc/df_ltrain.hip
Every wave of workgroups 0 and 128 stores s_memtime for its 32-sample steps (the first 31): 1 + 4k the step's
DMA wait and barrier passed, 2 + 4k split phase issued, 3 + 4k second barrier passed, 4 + 4k
MFMA phase issued; 0 kernel start, 127 after the partial-row stores.  Read back with
tools/ldense_stamps.py --ldw."""
import sys

BLOCK = '''#ifdef DF_LDW_STAMPS  // diagnostic build: s_memtime of each wave's phases in workgroups 0 and 128
__device__ uint64_t g_ldw_stamps[2 * 4 * 128];
#define DF_WST(ev) do { if ((blockIdx.x == 0 || blockIdx.x == 128) && (threadIdx.x & 63) == 0 && (ev) < 128) \\
    g_ldw_stamps[((blockIdx.x ? 1 : 0) * 4 + (threadIdx.x >> 6)) * 128 + (ev)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define DF_WST(ev) do {} while (0)
#endif
'''

ACCESSOR = '''
#ifdef DF_LDW_STAMPS
extern "C" int df_diag_ldw_stamps(uint64_t* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ldw_stamps), sizeof(g_ldw_stamps));
}
#endif
'''

EDITS = [  # (anchor, inserted before, inserted after)
    ("    [[maybe_unused]] f32x4 fr[2][2];\n    if (s_begin < s_end) {",
     "    DF_WST(0);\n    int kst = 0;\n", ""),
    ("        __syncthreads();                                     // ... every wave's; the planes are free\n",
     "", "        DF_WST(1 + 4 * kst);\n"),
    ("        __syncthreads();                                     // planes written; the stage is free\n",
     "        DF_WST(2 + 4 * kst);\n", "        DF_WST(3 + 4 * kst);\n"),
]


def main():
    path = sys.argv[1]
    s = open(path).read()
    anchor = '#include "df_train_impl.h"\n'
    assert s.count(anchor) == 1
    s = s.replace(anchor, anchor + "\n" + BLOCK, 1)
    for old, before, after in EDITS:
        assert s.count(old) == 1, old
        s = s.replace(old, before + old + after, 1)
    # end of the MFMA phase (the loop's last statement) and the kernel end
    old = ("                    acc[im][NI * hv + in] = uni::mfma_bf(wa[0], xb[in][0], v4);\n"
           "                }\n            }\n        }\n    }\n")
    assert s.count(old) == 1
    s = s.replace(old, old[:-len("    }\n")] + "        DF_WST(4 + 4 * kst);\n        ++kst;\n    }\n", 1)
    old = "        dst[a.b_off + tid] = ((dbl[tid] + dbl[256 + tid]) + dbl[512 + tid]) + dbl[768 + tid];\n}\n#else"
    assert s.count(old) == 1
    s = s.replace(old, old[:-len("}\n#else")] + "    DF_WST(127);\n}\n#else", 1)
    s = s.rstrip("\n") + "\n" + ACCESSOR
    open(path, "w").write(s)
    print("instrumented", path)


if __name__ == "__main__":
    main()
