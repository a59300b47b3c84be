// Probe: issue cost per wave of the MFMA shapes the headline kernel could use for its
// output Dense, calibrated against v_mfma_f32_16x16x4_f32.
// One workgroup of 4 waves per CU (one wave per SIMD), 8 independent accumulator chains per
// wave so dependency latency is hidden; time from hipEvents over the whole grid.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kIters = 65536, kChains = 8;

__global__ void __launch_bounds__(256) mfma_4x4(const float* in, float* out) {
    const float a = in[threadIdx.x & 63], b = in[(threadIdx.x + 7) & 63];
    f32x4 c[kChains];
    for (int j = 0; j < kChains; ++j) c[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < kChains; ++j) c[j] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[j], 0, 0, 0);
    float s = 0.f;
    for (int j = 0; j < kChains; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) mfma_16x16x4(const float* in, float* out) {
    const float a = in[threadIdx.x & 63], b = in[(threadIdx.x + 7) & 63];
    f32x4 c[kChains];
    for (int j = 0; j < kChains; ++j) c[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < kChains; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[j], 0, 0, 0);
    float s = 0.f;
    for (int j = 0; j < kChains; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Inline asm, 4 chains: through the builtin the compiler shuffles the accumulators with AGPR moves
// inside the loop.
constexpr int kChainsBf16 = 4;
__global__ void __launch_bounds__(256) mfma_16x16x32_bf16(const float* in, float* out) {
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
        a[e] = (__bf16)in[(threadIdx.x + e) & 63];
        b[e] = (__bf16)in[(threadIdx.x + 3 * e) & 63];
    }
    f32x4 c[kChainsBf16];
    for (int j = 0; j < kChainsBf16; ++j) c[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < kChainsBf16; ++j)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c[j]) : "v"(a), "v"(b));
    float s = 0.f;
    for (int j = 0; j < kChainsBf16; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) valu_fmac(const float* in, float* out) {
    const float a = in[threadIdx.x & 63], b = in[(threadIdx.x + 7) & 63];
    float c[kChains * 4];
    for (int j = 0; j < kChains * 4; ++j) c[j] = a * (float)(j + 1);  // no loads: their waitcnts would sit in the loop
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < kChains * 4; ++j) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(c[j]) : "v"(a), "v"(b));
    float s = 0.f;
    for (int j = 0; j < kChains * 4; ++j) s += c[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
static float time_ms(K kern, int grid, const float* in, float* out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out);
    hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0); hipEventDestroy(e1);
    return ms / 5.f;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    float *in, *out;
    hipMalloc(&in, 64 * 4);
    hipMalloc(&out, (size_t)cus * 2 * 256 * 4);
    float h[64];
    for (int i = 0; i < 64; ++i) h[i] = 1e-3f * (i + 1);
    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    for (int waves = 1; waves <= 2; ++waves) {
        // waves per SIMD: one 4-wave workgroup per CU, or two.
        const int grid = cus * waves;
        // Instructions per SIMD: waves * kIters * kChains (x4 for the VALU kernel).
        const double per_simd = (double)waves * kIters * kChains;
        // Clock from the shape whose rate the f32 MFMA peak fixes: 157.3 TF / (1024 SIMDs x 2.4 GHz)
        // = 64 FLOP per SIMD cycle, so v_mfma_f32_16x16x4_f32 (2048 FLOP) issues every 32 cycles.
        const double t_16x16x4 = time_ms(mfma_16x16x4, grid, in, out) / per_simd;
        const double cyc = 32.0 / t_16x16x4;  // cycles per ms
        struct { const char* name; double ms, n; } r[] = {
            {"v_fmac_f32", time_ms(valu_fmac, grid, in, out), per_simd * 4},
            {"v_mfma_f32_4x4x1_16b_f32", time_ms(mfma_4x4, grid, in, out), per_simd},
            {"v_mfma_f32_16x16x4_f32 (calibration, 32)", t_16x16x4 * per_simd, per_simd},
            {"v_mfma_f32_16x16x32_bf16", time_ms(mfma_16x16x32_bf16, grid, in, out), per_simd * kChainsBf16 / kChains},
        };
        printf("CUs %d, %d wave(s) per SIMD, clock (from the 16x16x4 f32 calibration) %.0f MHz\n", cus,
               waves, cyc / 1e3);
        for (auto& x : r)
            printf("  %-40s %8.4f ms  %6.2f SIMD cycles per wave instruction\n", x.name, x.ms, x.ms / x.n * cyc);
    }
    return 0;
}
