// Probe: does a partner wave's VALU stream slow a wave's MFMA stream on the same SIMD?
// One 8-wave workgroup per CU (two waves per SIMD): waves 0-3 issue back-to-back
// v_mfma_f32_16x16x32_bf16 (two accumulator chains), waves 4-7 issue a VALU-only stream of
// one instruction kind; s_memtime around each wave's loop.  Cycles per 12 MFMAs of the
// MFMA waves (median), against the partner kinds (none: waves 4-7 exit at once).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/mfma_pair tools/probe/mfma_pair.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kIters = 4096;

#define M12                                               \
    "v_mfma_f32_16x16x32_bf16 %[c0], %[a], %[b], %[c0]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c1], %[a], %[b], %[c1]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c0], %[a], %[b], %[c0]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c1], %[a], %[b], %[c1]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c0], %[a], %[b], %[c0]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c1], %[a], %[b], %[c1]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c0], %[a], %[b], %[c0]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c1], %[a], %[b], %[c1]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c0], %[a], %[b], %[c0]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c1], %[a], %[b], %[c1]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c0], %[a], %[b], %[c0]\n\t" \
    "v_mfma_f32_16x16x32_bf16 %[c1], %[a], %[b], %[c1]"

#define V4(I) I " %[f0], %[f0], %[x]\n\t" I " %[f1], %[f1], %[x]\n\t" I " %[f2], %[f2], %[x]\n\t" I " %[f3], %[f3], %[x]"

template <int KIND>
__global__ void __launch_bounds__(512) pair(const float* in, float* out, unsigned long long* cyc) {
    const int wave = threadIdx.x >> 6;
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
        a[e] = (__bf16)in[(threadIdx.x + e) & 63];
        b[e] = (__bf16)in[(threadIdx.x + 3 * e) & 63];
    }
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
    float f0 = in[1], f1 = in[2], f2 = in[3], f3 = in[4];
    f32x2 p0 = {in[5], in[6]}, p1 = {in[7], in[8]};
    const float x = in[9];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave < 4) {
        for (int i = 0; i < kIters; ++i)
            asm volatile(M12 : [c0] "+v"(c0), [c1] "+v"(c1) : [a] "v"(a), [b] "v"(b));
    } else if (KIND == 1) {  // v_add_f32, 48 per iteration (the MFMA waves' 12 MFMAs ≈ 196 cycles)
        for (int i = 0; i < kIters; ++i)
            asm volatile(V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t"
                         V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t"
                         V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t" V4("v_add_f32") "\n\t" V4("v_add_f32")
                         : [f0] "+v"(f0), [f1] "+v"(f1), [f2] "+v"(f2), [f3] "+v"(f3) : [x] "v"(x));
    } else if (KIND == 2) {  // v_dot2c_f32_bf16, 16 per iteration
        for (int i = 0; i < kIters; ++i)
            asm volatile(V4("v_dot2c_f32_bf16") "\n\t" V4("v_dot2c_f32_bf16") "\n\t" V4("v_dot2c_f32_bf16") "\n\t"
                         V4("v_dot2c_f32_bf16")
                         : [f0] "+v"(f0), [f1] "+v"(f1), [f2] "+v"(f2), [f3] "+v"(f3) : [x] "v"(x));
    } else if (KIND == 3) {  // v_pk_add_f32, 16 per iteration
        for (int i = 0; i < kIters; ++i)
            asm volatile(
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]\n\t"
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]\n\t"
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]\n\t"
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]\n\t"
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]\n\t"
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]\n\t"
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]\n\t"
                "v_pk_add_f32 %[p0], %[p0], %[p1]\n\tv_pk_add_f32 %[p1], %[p1], %[p0]"
                : [p0] "+v"(p0), [p1] "+v"(p1));
    } else if (KIND == 4) {  // v_cvt_pk_bf16_f32, 48 per iteration
        for (int i = 0; i < kIters; ++i)
            asm volatile(V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32") "\n\t"
                         V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32") "\n\t"
                         V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32") "\n\t"
                         V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32") "\n\t" V4("v_cvt_pk_bf16_f32")
                         : [f0] "+v"(f0), [f1] "+v"(f1), [f2] "+v"(f2), [f3] "+v"(f3) : [x] "v"(x));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = c0[0] + c1[0] + f0 + f1 + f2 + f3 + p0[0] + p1[1];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

typedef void (*K)(const float*, float*, unsigned long long*);

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    float *in, *out;
    unsigned long long* cyc;
    (void)hipMalloc(&in, 64 * 4);
    (void)hipMalloc(&out, (size_t)cus * 512 * 4);
    (void)hipMalloc(&cyc, (size_t)cus * 8 * 8);
    float h[64];
    for (int i = 0; i < 64; ++i) h[i] = 1e-3f * (i + 1);
    (void)hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    std::vector<unsigned long long> hc((size_t)cus * 8);
    K ks[] = {pair<0>, pair<1>, pair<2>, pair<3>, pair<4>};
    const char* names[] = {"partner idle", "partner 48 v_add_f32", "partner 16 v_dot2c_f32_bf16",
                           "partner 16 v_pk_add_f32", "partner 48 v_cvt_pk_bf16_f32"};
    for (int v = 0; v < 5; ++v) {
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(ks[v], dim3(cus), dim3(512), 0, 0, in, out, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hc.data(), cyc, hc.size() * 8, hipMemcpyDeviceToHost);
        std::vector<unsigned long long> m, vv;
        for (int b = 0; b < cus; ++b)
            for (int w = 0; w < 8; ++w) (w < 4 ? m : vv).push_back(hc[b * 8 + w]);
        std::sort(m.begin(), m.end());
        std::sort(vv.begin(), vv.end());
        printf("%-34s MFMA waves %7.1f cycles per 12 MFMAs, partner waves %7.1f cycles per iteration\n", names[v],
               (double)m[m.size() / 2] / kIters, (double)vv[vv.size() / 2] / kIters);
        fflush(stdout);
    }
    return 0;
}
