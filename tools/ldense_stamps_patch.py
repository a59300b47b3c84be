"""Instrument df_ltrain.hip in place with the phase stamps tools/ldense_stamps.py reads
(diagnostic only; the product source carries no stamps, so its hash is unchanged):
    python tools/ldense_stamps_patch.py densityflows.jl_amd/csrc/df_ltrain.hip [second_wg]
    OBJS=df_ltrain bash tools/build_variant.sh lst "-DDF_LDENSE_STAMPS"
    git checkout densityflows.jl_amd/csrc/df_ltrain.hip
Every wave of workgroups 0 and `second_wg` (default 128) of each ldense_kernel launch stores
s_memtime at the events listed in tools/ldense_stamps.py."""
import sys

BLOCK = '''#ifdef DF_LDENSE_STAMPS  // diagnostic build: s_memtime of each wave's phases in workgroups 0 and {wg}
__device__ uint64_t g_ldense_stamps[2 * 8 * 128];
#define DF_LST(ev) do {{ if ((blockIdx.x == 0 || blockIdx.x == {wg}) && (threadIdx.x & 63) == 0) \\
    g_ldense_stamps[((blockIdx.x ? 1 : 0) * 8 + (threadIdx.x >> 6)) * 128 + (ev)] = __builtin_amdgcn_s_memtime(); }} while (0)
#else
#define DF_LST(ev) do {{}} while (0)
#endif
'''

ACCESSOR = '''
#ifdef DF_LDENSE_STAMPS
extern "C" int df_diag_ldense_stamps(uint64_t* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ldense_stamps), sizeof(g_ldense_stamps));
}
#endif
'''

# (anchor text, text inserted before it)
EDITS = [
    ("    for (int64_t r = 0; r < rounds; ++r) {\n        const int64_t t0 = ((r * gridDim.x + blockIdx.x) * NW + wave) * T;",
     "    DF_LST(0);\n"),
    ("        const int64_t t0 = ((r * gridDim.x + blockIdx.x) * NW + wave) * T;",
     "        DF_LST(1 + 24 * (int)r);\n"),
    ("                    if (i + 1 < total) dma((int)((i + 1) % nchunks), smem + (((i + 1) & 1) ? chunk_bytes : 0));\n"
     "                    buf = smem + ((i & 1) ? chunk_bytes : 0);\n                }\n                uni::bf16x8 xp[T][3];",
     "                    DF_LST(2 + 24 * (int)r + c);\n"),
    ("        if constexpr (EPI == LEPI_DACT || XB) {\n#if DF_LDENSE_DIAG == 1",
     "        DF_LST(10 + 24 * (int)r);\n"),
    ("                if constexpr (XB && DF_LDENSE_ZV_EARLY) load_zv();",
     "                DF_LST(12 + 24 * (int)r + 4 * t);\n"),
    ("                if constexpr (XB) {\n                    // x̄ = W0ᵀ δ0",
     "                DF_LST(13 + 24 * (int)r + 4 * t);\n"),
    ("#pragma unroll\n                    for (int m = 0; m < 4; ++m)\n#pragma unroll\n                        for (int q = 0; q < 4; ++q)\n"
     "                            if (m < a.w0t_mt && valid[t]) {",
     "                    DF_LST(14 + 24 * (int)r + 4 * t);\n"),
]


def main():
    path = sys.argv[1]
    wg = sys.argv[2] if len(sys.argv) > 2 else "128"
    s = open(path).read()
    anchor = '#include "df_train_impl.h"\n'
    assert s.count(anchor) == 1
    s = s.replace(anchor, anchor + "\n" + BLOCK.format(wg=wg), 1)
    for old, ins in EDITS:
        assert s.count(old) == 1, old
        s = s.replace(old, ins + old, 1)
    # after the z̄ stores of a tile, at the end of each round, after the final drain
    old = ("                                if (c != 0xffu) a.zbar[s * a.d + c] = zv[m][q] + xb[m][q];\n"
           "                            }\n                }")
    assert s.count(old) == 1
    s = s.replace(old, old[:-len("                }")] + "                    DF_LST(15 + 24 * (int)r + 4 * t);\n                }", 1)
    old = "            }\n        }\n    }\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n}\n"
    assert s.count(old) == 1
    s = s.replace(old, "            }\n        }\n        DF_LST(11 + 24 * (int)r);\n    }\n"
                  "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    DF_LST(120);\n}\n", 1)
    s = s.rstrip("\n") + "\n" + ACCESSOR
    open(path, "w").write(s)
    print("instrumented", path)


if __name__ == "__main__":
    main()
