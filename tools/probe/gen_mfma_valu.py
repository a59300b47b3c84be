"""Generate tools/probe/mfma_valu.hip: cycles per loop iteration of a fixed instruction
sequence of 12 v_mfma_f32_16x16x32_bf16 with VALU fillers placed between them, one wave per
SIMD (one 4-wave workgroup per CU), timed with s_memtime around the loop.  Each variant is
ONE inline-asm statement, so the order below is the issued order.
    python tools/probe/gen_mfma_valu.py && hipcc --offload-arch=gfx950 -O3 \
        -o tools/probe/mfma_valu tools/probe/mfma_valu.hip
"""
import os

M = "v_mfma_f32_16x16x32_bf16 {c}, %[a], %[b], {c}"


def mf(i, order):
    return M.format(c="%[c" + str(order(i)) + "]")


def alt(i):
    return i & 1          # two chains alternating


def seq(i):
    return i // 6         # chain 0 six times, then chain 1


def ind(i):
    return i              # 12 independent accumulators


V = {
    "add": "v_add_f32 %[f{k}], %[f{k}], %[x]",
    "adddep": "v_add_f32 %[f0], %[f0], %[x]",
    "cvt": "v_cvt_pk_bf16_f32 %[f{k}], %[f{k}], %[x]",
    "dot2": "v_dot2c_f32_bf16 %[f{k}], %[f{k}], %[x]",
    "sub": "v_sub_f32 %[f{k}], %[f{k}], %[x]",
    "shl": "v_lshlrev_b32 %[f{k}], 16, %[f{k}]",
    "max": "v_max_i32 %[f{k}], 0, %[f{k}]",
    "pkadd": "v_pk_add_f32 %[p{k}], %[p{k}], %[p{k}]",
    "pkfma": "v_pk_fma_f32 %[p{k}], %[p{k}], %[p{k}], %[p{k}]",
    "accr": "v_accvgpr_read_b32 %[f{k}], %[g{k}]",
    "accw": "v_accvgpr_write_b32 %[g{k}], %[f{k}]",
    "fmac": "v_fmac_f32 %[f{k}], %[x], %[x]",
    "mov": "v_mov_b32 %[f{k}], %[x]",
    "cnd": "v_cndmask_b32 %[f{k}], %[f{k}], %[x], vcc",
    "pl16": "v_permlane16_swap_b32 %[f{k}], %[h{k}]",
    "exp": "v_exp_f32 %[f{k}], %[f{k}]",
    "cvtf": "v_cvt_f32_bf16 %[f{k}], %[f{k}]",
    "and": "v_and_b32 %[f{k}], 0xffff0000, %[f{k}]",
    "salu": "s_add_u32 %[s{k}], %[s{k}], 1",
}

# (name, chain order, accumulators, per-gap filler kinds, block filler kinds after the MFMAs)
VARIANTS = [
    ("alt, no VALU", alt, 2, [], []),
    ("seq (dependent back to back), no VALU", seq, 2, [], []),
    ("ind (12 accumulators), no VALU", ind, 12, [], []),
    ("alt + 1 v_add per gap", alt, 2, ["add"], []),
    ("alt + 2 v_add per gap", alt, 2, ["add", "add"], []),
    ("alt + 3 v_add per gap", alt, 2, ["add", "add", "add"], []),
    ("alt + 12 v_add as a block", alt, 2, [], ["add"] * 12),
    ("alt + 24 v_add as a block", alt, 2, [], ["add"] * 24),
    ("alt + 1 dependent v_add per gap", alt, 2, ["adddep"], []),
    ("alt + 1 v_cvt_pk_bf16_f32 per gap", alt, 2, ["cvt"], []),
    ("alt + 1 v_dot2c_f32_bf16 per gap", alt, 2, ["dot2"], []),
    ("alt + 12 v_dot2c as a block", alt, 2, [], ["dot2"] * 12),
    ("alt + 1 v_sub_f32 per gap", alt, 2, ["sub"], []),
    ("alt + 1 v_lshlrev_b32 per gap", alt, 2, ["shl"], []),
    ("alt + 1 v_max_i32 per gap", alt, 2, ["max"], []),
    ("alt + 1 v_pk_add_f32 per gap", alt, 2, ["pkadd"], []),
    ("seq + 1 v_add per gap", seq, 2, ["add"], []),
    ("ind + 1 v_add per gap", ind, 12, ["add"], []),
    ("ind + 2 v_add per gap", ind, 12, ["add", "add"], []),
    ("alt + v_add in every 2nd gap", alt, 2, ["add@2"], []),
    ("alt + 1 v_pk_fma_f32 per gap", alt, 2, ["pkfma"], []),
    ("alt + 1 v_accvgpr_read per gap", alt, 2, ["accr"], []),
    ("alt + 1 v_accvgpr_write per gap", alt, 2, ["accw"], []),
    ("alt + 12 v_accvgpr_read as a block", alt, 2, [], ["accr"] * 12),
    ("alt + 1 v_fmac_f32 per gap", alt, 2, ["fmac"], []),
    ("alt + 2 v_fmac_f32 per gap", alt, 2, ["fmac", "fmac"], []),
    ("alt + 1 v_mov_b32 per gap", alt, 2, ["mov"], []),
    ("alt + 1 v_cndmask per gap", alt, 2, ["cnd"], []),
    ("alt + 1 v_permlane16_swap per gap", alt, 2, ["pl16"], []),
    ("alt + 1 v_exp_f32 per gap", alt, 2, ["exp"], []),
    ("alt + 1 v_cvt_f32_bf16 per gap", alt, 2, ["cvtf"], []),
    ("alt + 1 v_and_b32 (literal) per gap", alt, 2, ["and"], []),
    ("alt + 2 s_add_u32 per gap", alt, 2, ["salu", "salu"], []),
    ("alt + 4 s_add_u32 per gap", alt, 2, ["salu"] * 4, []),
    ("alt + 1 v_add + 1 s_add per gap", alt, 2, ["add", "salu"], []),
    ("AGPR alt, no VALU", alt, 2, [], [], "a"),
    ("AGPR alt + 1 v_add per gap", alt, 2, ["add"], [], "a"),
    ("AGPR alt + 2 v_add per gap", alt, 2, ["add", "add"], [], "a"),
    ("AGPR alt + 12 v_add as a block", alt, 2, [], ["add"] * 12, "a"),
    ("AGPR seq + 1 v_add per gap", seq, 2, ["add"], [], "a"),
]


def body(order, nacc, gap, block):
    lines, k = [], 0
    for i in range(12):
        lines.append(mf(i, order))
        for g in gap:
            if g.endswith("@2"):
                if i % 2:
                    continue
                g = g[:-2]
            lines.append(V[g].format(k=k % 12))
            k += 1
    for g in block:
        lines.append(V[g].format(k=k % 12))
        k += 1
    return "\\n\\t".join(lines)


def kernel(idx, name, order, nacc, gap, block, ak="v"):
    accs = ", ".join("[c%d] \"+%s\"(c[%d])" % (j, ak, j) for j in range(nacc))
    fills = ", ".join("[f%d] \"+v\"(f[%d])" % (j, j) for j in range(12))
    kinds = gap + block
    pk = ", ".join("[p%d] \"+v\"(p[%d])" % (j, j) for j in range(12)) if any("pk" in g for g in kinds) else ""
    ag = ", ".join("[g%d] \"+a\"(gg[%d])" % (j, j) for j in range(12)) if any(g in ("accr", "accw") for g in kinds) else ""
    hh = ", ".join("[h%d] \"+v\"(hh[%d])" % (j, j) for j in range(12)) if "pl16" in kinds else ""
    ss = ", ".join("[s%d] \"+s\"(ss[%d])" % (j, j) for j in range(12)) if "salu" in kinds else ""
    ops = accs + ", " + fills + "".join(", " + x for x in (pk, ag, hh, ss) if x)
    return f'''
// {name}
__global__ void __launch_bounds__(256) k{idx}(const float* in, float* out, unsigned long long* cyc) {{
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {{ a[e] = (__bf16)in[(threadIdx.x + e) & 63]; b[e] = (__bf16)in[(threadIdx.x + 3 * e) & 63]; }}
    f32x4 c[{nacc}];
    for (int j = 0; j < {nacc}; ++j) c[j] = f32x4{{0.f, 0.f, 0.f, 0.f}};
    float f[12];
    for (int j = 0; j < 12; ++j) f[j] = in[j];
    [[maybe_unused]] f32x2 p[12];
    for (int j = 0; j < 12; ++j) p[j] = f32x2{{in[j], in[j + 1]}};
    const float x = in[40];
    [[maybe_unused]] float gg[12], hh[12];
    [[maybe_unused]] unsigned ss[12];
    for (int j = 0; j < 12; ++j) {{ gg[j] = in[j + 20]; hh[j] = in[j + 30]; ss[j] = j; }}
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i)
        asm volatile("{body(order, nacc, gap, block)}" : {ops} : [a] "v"(a), [b] "v"(b), [x] "v"(x) : "scc", "vcc");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int j = 0; j < {nacc}; ++j) s += c[j][0];
    for (int j = 0; j < 12; ++j) s += f[j] + p[j][0] + gg[j] + hh[j] + (float)ss[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}}
'''


def main():
    src = ['// Generated by tools/probe/gen_mfma_valu.py — do not edit.',
           '#include <hip/hip_runtime.h>', '#include <algorithm>', '#include <cstdio>', '#include <vector>',
           'typedef float f32x4 __attribute__((ext_vector_type(4)));',
           'typedef float f32x2 __attribute__((ext_vector_type(2)));',
           'typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));',
           'constexpr int kIters = 4096;']
    for i, v in enumerate(VARIANTS):
        src.append(kernel(i, *v))
    src.append('typedef void (*K)(const float*, float*, unsigned long long*);')
    src.append('int main() {')
    src.append('    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0); const int cus = p.multiProcessorCount;')
    src.append('    float *in, *out; unsigned long long* cyc;')
    src.append('    hipMalloc(&in, 64 * 4); hipMalloc(&out, (size_t)cus * 256 * 4); hipMalloc(&cyc, (size_t)cus * 4 * 8);')
    src.append('    float h[64]; for (int i = 0; i < 64; ++i) h[i] = 1e-3f * (i + 1);')
    src.append('    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);')
    src.append('    std::vector<unsigned long long> hc((size_t)cus * 4);')
    ks = ", ".join("k%d" % i for i in range(len(VARIANTS)))
    names = ", ".join('"%s"' % v[0] for v in VARIANTS)
    src.append('    K ks[] = {%s};' % ks)
    src.append('    const char* names[] = {%s};' % names)
    src.append('    for (int v = 0; v < %d; ++v) {' % len(VARIANTS))
    src.append('        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(ks[v], dim3(cus), dim3(256), 0, 0, in, out, cyc);')
    src.append('        hipDeviceSynchronize();')
    src.append('        hipMemcpy(hc.data(), cyc, hc.size() * 8, hipMemcpyDeviceToHost);')
    src.append('        std::sort(hc.begin(), hc.end());')
    src.append('        printf("%-45s %7.1f cycles per 12 MFMAs (median wave)\\n", names[v], (double)hc[hc.size() / 2] / kIters);')
    src.append('        fflush(stdout);')
    src.append('    }')
    src.append('    return 0;')
    src.append('}')
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mfma_valu.hip")
    open(out, "w").write("\n".join(src) + "\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
