// Probe: is v_dot2c_f32_bf16(h, {-1, 0}, x) == x - (float)h bitwise on gfx950, where
// h = RNE bf16 pair of (x0, x1)?  (The SPLIT kernels' remainder r = x - hi without
// the two bf16 → f32 unpacks.)  Checks both remainder levels of the bf16x3 split over
// 2^24 values per pass: random magnitudes over the normal f32 range, relu outputs,
// values near bf16 ties, tiny values near the denormal range.
#include <hip/hip_runtime.h>
#include "df_uniform_impl.h"  // the kernels' own split helper (df::uni::split2)
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cstdlib>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int OPAQUE>
__global__ void k(uint32_t seed, int pass, unsigned long long* bad, uint32_t* example) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t u0 = hash(i * 2 + seed), u1 = hash(i * 2 + 1 + seed * 7919u);
    if (pass == 1) { u0 = (u0 & 0x807fffffu) | (((u0 >> 23) % 40 + 107) << 23); u1 = (u1 & 0x807fffffu) | (((u1 >> 23) % 40 + 107) << 23); }
    if (pass == 2) { u0 = (u0 & 0x807f0000u) | 0x8000u | (120u << 23); u1 = (u1 & 0xff7fffffu); }  // bf16 ties
    if (pass == 3) { u0 = (u0 & 0x807fffffu) | ((1 + (u0 >> 23) % 30) << 23); u1 = (u1 & 0x807fffffu) | ((1 + (u1 >> 23) % 30) << 23); }
    float x0 = __uint_as_float(u0), x1 = __uint_as_float(u1);
    // inf / nan, and |x| that rounds to a bf16 inf (≥ 0x7f7f8000): the pair's other
    // product is then 0·inf = NaN (activations of that size have overflowed already)
    if ((u0 & 0x7fffffffu) >= 0x7f7f8000u || (u1 & 0x7fffffffu) >= 0x7f7f8000u) return;
    if (pass == 1) { x0 = fmaxf(x0, 0.f); x1 = fmaxf(x1, 0.f); }
    bf16x2 n0 = {(__bf16)-1.0f, (__bf16)0.0f};
    bf16x2 n1 = {(__bf16)0.0f, (__bf16)-1.0f};
    if (OPAQUE) {  // the constants through VGPRs (no inline-constant encoding)
        uint32_t c0 = 0x0000bf80u, c1 = 0xbf800000u;
        asm volatile("" : "+v"(c0), "+v"(c1));
        n0 = __builtin_bit_cast(bf16x2, c0);
        n1 = __builtin_bit_cast(bf16x2, c1);
    }
    const bf16x2 h = {(__bf16)x0, (__bf16)x1};
    const float r0 = x0 - (float)h[0], r1 = x1 - (float)h[1];
    const float d0 = __builtin_amdgcn_fdot2_f32_bf16(h, n0, x0, false);
    const float d1 = __builtin_amdgcn_fdot2_f32_bf16(h, n1, x1, false);
    const bf16x2 m = {(__bf16)r0, (__bf16)r1};
    const float l0 = r0 - (float)m[0], l1 = r1 - (float)m[1];
    const float e0 = __builtin_amdgcn_fdot2_f32_bf16(m, n0, r0, false);
    const float e1 = __builtin_amdgcn_fdot2_f32_bf16(m, n1, r1, false);
    const bool ok = __float_as_uint(d0) == __float_as_uint(r0) && __float_as_uint(d1) == __float_as_uint(r1) &&
                    __float_as_uint(e0) == __float_as_uint(l0) && __float_as_uint(e1) == __float_as_uint(l1);
    if (!ok) {
        if (atomicAdd(bad, 1ull) == 0) {
            example[0] = u0; example[1] = u1;
            example[2] = __float_as_uint(r0); example[3] = __float_as_uint(d0);
            example[4] = __float_as_uint(l0); example[5] = __float_as_uint(e0);
        }
    }
}

// The product helper itself: df::uni::split2's planes (HELPER = 1) against the plain
// RNE split (HELPER = 0), each written to memory by its own kernel and compared on the
// host (no cross-kernel folding of the two computations).
__device__ __forceinline__ void probe_inputs(uint32_t i, uint32_t seed, int pass, float& x0, float& x1, bool& skip) {
    uint32_t u0 = hash(i * 2 + seed), u1 = hash(i * 2 + 1 + seed * 7919u);
    if (pass == 1) { u0 = (u0 & 0x807fffffu) | (((u0 >> 23) % 40 + 107) << 23); u1 = (u1 & 0x807fffffu) | (((u1 >> 23) % 40 + 107) << 23); }
    if (pass == 2) { u0 = (u0 & 0x807f0000u) | 0x8000u | (120u << 23); u1 = (u1 & 0xff7fffffu); }
    if (pass == 3) { u0 = (u0 & 0x807fffffu) | ((1 + (u0 >> 23) % 30) << 23); u1 = (u1 & 0x807fffffu) | ((1 + (u1 >> 23) % 30) << 23); }
    skip = (u0 & 0x7fffffffu) >= 0x7f7f8000u || (u1 & 0x7fffffffu) >= 0x7f7f8000u;
    x0 = __uint_as_float(u0);
    x1 = __uint_as_float(u1);
    if (pass == 1) { x0 = fmaxf(x0, 0.f); x1 = fmaxf(x1, 0.f); }
}

template <int HELPER>
__global__ void k_planes(uint32_t seed, int pass, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    float x0, x1;
    bool skip;
    probe_inputs(i, seed, pass, x0, x1, skip);
    uint32_t w[3] = {0u, 0u, 0u};
    if (!skip) {
        if (HELPER) {
            df::uni::bf16x2 p0, p1, p2;
            df::uni::split2(x0, x1, p0, p1, p2);
            w[0] = __builtin_bit_cast(uint32_t, p0);
            w[1] = __builtin_bit_cast(uint32_t, p1);
            w[2] = __builtin_bit_cast(uint32_t, p2);
        } else {
            const float x[2] = {x0, x1};
            for (int e = 0; e < 2; ++e) {
                const __bf16 h = (__bf16)x[e];
                const float r = x[e] - (float)h;
                const __bf16 m = (__bf16)r;
                const __bf16 l = (__bf16)(r - (float)m);
                w[0] |= (uint32_t)__builtin_bit_cast(uint16_t, h) << (16 * e);
                w[1] |= (uint32_t)__builtin_bit_cast(uint16_t, m) << (16 * e);
                w[2] |= (uint32_t)__builtin_bit_cast(uint16_t, l) << (16 * e);
            }
        }
    }
    out[3 * i] = w[0];
    out[3 * i + 1] = w[1];
    out[3 * i + 2] = w[2];
}

// The matrix-pipe remainders (df::uni::split8_mrem, DF_SPLIT_MREM): each lane's 8
// values as two accumulator tiles, planes written per pair in the k_planes layout.
// Non-finite inputs are zeroed first (0·inf in the −I product would poison the column;
// such activations have overflowed already), and their planes reported as 0.
__global__ void k_planes_mrem(uint32_t seed, int pass, uint32_t* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    float v[8];
    bool sk[4];
    for (int q = 0; q < 4; ++q) {
        float x0, x1;
        probe_inputs(4 * t + q, seed, pass, x0, x1, sk[q]);
        v[2 * q] = sk[q] ? 0.f : x0;
        v[2 * q + 1] = sk[q] ? 0.f : x1;
    }
    const df::f32x4 a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
    df::uni::bf16x8 p[3];
    df::uni::split8_mrem(df::uni::neg_eye(), a, b, p[0], p[1], p[2]);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
        const u32x4 w = __builtin_bit_cast(u32x4, p[pl]);   // dword q = elements (2q, 2q+1)
#pragma unroll
        for (int q = 0; q < 4; ++q) out[3 * (4 * t + q) + pl] = sk[q] ? 0u : w[q];
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* ex;
    hipMalloc(&bad, 8);
    hipMalloc(&ex, 32);
    int rc = 0;
    const char* names[] = {"random normal f32", "relu outputs 2^-20..2^20", "bf16 ties", "near-denormal"};
    for (int opq = 0; opq < 2; ++opq)
    for (int pass = 0; pass < 4; ++pass) {
        unsigned long long nb = 0;
        uint32_t e[6] = {0, 0, 0, 0, 0, 0};
        hipMemset(bad, 0, 8);
        hipMemset(ex, 0, 32);
        if (opq) hipLaunchKernelGGL(k<1>, dim3(1 << 16), dim3(256), 0, 0, 1234u + pass, pass, bad, ex);
        else hipLaunchKernelGGL(k<0>, dim3(1 << 16), dim3(256), 0, 0, 1234u + pass, pass, bad, ex);
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(e, ex, 24, hipMemcpyDeviceToHost);
        printf("%s %-28s mismatches %llu of 2^24", opq ? "vgpr-const   " : "inline-const ", names[pass], nb);
        if (nb) printf("  e.g. x0=%08x x1=%08x r0=%08x dot=%08x l0=%08x dot=%08x", e[0], e[1], e[2], e[3], e[4], e[5]);
        printf("\n");
        if (nb && opq) rc = 1;
    }
    const size_t np = (size_t)1 << 24, nb = 3 * np * sizeof(uint32_t);
    uint32_t *dh, *dp;
    hipMalloc(&dh, nb);
    hipMalloc(&dp, nb);
    uint32_t* hh = (uint32_t*)malloc(nb);
    uint32_t* hp = (uint32_t*)malloc(nb);
    for (int pass = 0; pass < 4; ++pass) {
        hipLaunchKernelGGL(k_planes<1>, dim3(np / 256), dim3(256), 0, 0, 1234u + pass, pass, dh);
        hipLaunchKernelGGL(k_planes<0>, dim3(np / 256), dim3(256), 0, 0, 1234u + pass, pass, dp);
        hipMemcpy(hh, dh, nb, hipMemcpyDeviceToHost);
        hipMemcpy(hp, dp, nb, hipMemcpyDeviceToHost);
        size_t bad_pairs = 0, first = 0;
        for (size_t i = 0; i < np; ++i)
            if (memcmp(hh + 3 * i, hp + 3 * i, 12) != 0) { if (!bad_pairs) first = i; ++bad_pairs; }
        printf("split2 helper %-28s mismatches %zu of 2^24", names[pass], bad_pairs);
        if (bad_pairs) printf("  e.g. pair %zu: helper %08x %08x %08x plain %08x %08x %08x", first, hh[3 * first],
                              hh[3 * first + 1], hh[3 * first + 2], hp[3 * first], hp[3 * first + 1], hp[3 * first + 2]);
        printf("\n");
        if (bad_pairs) rc = 1;
    }
    for (int pass = 0; pass < 4; ++pass) {   // the matrix-pipe form against the plain split
        hipLaunchKernelGGL(k_planes_mrem, dim3(np / 4 / 256), dim3(256), 0, 0, 1234u + pass, pass, dh);
        hipLaunchKernelGGL(k_planes<0>, dim3(np / 256), dim3(256), 0, 0, 1234u + pass, pass, dp);
        hipMemcpy(hh, dh, nb, hipMemcpyDeviceToHost);
        hipMemcpy(hp, dp, nb, hipMemcpyDeviceToHost);
        size_t bad_pairs = 0, first = 0;
        for (size_t i = 0; i < np; ++i)
            if (memcmp(hh + 3 * i, hp + 3 * i, 12) != 0) { if (!bad_pairs) first = i; ++bad_pairs; }
        printf("split8 mrem   %-28s mismatches %zu of 2^24", names[pass], bad_pairs);
        if (bad_pairs) printf("  e.g. pair %zu: mrem %08x %08x %08x plain %08x %08x %08x", first, hh[3 * first],
                              hh[3 * first + 1], hh[3 * first + 2], hp[3 * first], hp[3 * first + 1], hp[3 * first + 2]);
        printf("\n");
        if (bad_pairs) rc = 1;
    }
    free(hh);
    free(hp);
    hipFree(dh);
    hipFree(dp);
    hipFree(bad);
    hipFree(ex);
    return rc;
}
