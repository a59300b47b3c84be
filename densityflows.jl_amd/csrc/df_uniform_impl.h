// df_uniform_impl.h — the specialised fused kernel for chains whose coupling
// layers all use the reference's default conditioner shape (_dflt_net,
// src/Layers.jl:33-50): Dense(in, H, σ), nh × Dense(H, H, σ), Dense(H, out),
// with H = 16·HT exactly, in <= 16, and each net resident in ONE LDS stage.
// Same numerics and data flow as the generic kernel (df_chain_impl.h) with
// every width known at compile time: no per-tile guards, ping-pong
// accumulators instead of register copies, compact per-net descriptors.
#pragma once

#include <type_traits>

#include "df_chain_impl.h"

namespace df {
namespace uni {


using impl::lds4;
using impl::mfma4;
using impl::Stager;

// relu(x) = max(0, x) as ONE v_max_i32 on the bit pattern: non-negative floats
// order like their integer images; negative floats (and -0) map to +0; a NaN
// with the sign bit clear (the canonical quiet NaN) propagates as in Julia.
__device__ __forceinline__ float relu_fast(float x) {
    return __int_as_float(__builtin_elementwise_max(__float_as_int(x), 0));
}

// Σ over the 4 lane groups of a wave (lanes l, l^16, l^32, l^48) without LDS:
// gfx950 v_permlane16_swap / v_permlane32_swap.  Every lane gets the bitwise
// identical total ((p0+p1)+(p2+p3), commutations only).
__device__ __forceinline__ float xgroup_sum(float p) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(p), __float_as_uint(p), false, false);
    const float q = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(q), __float_as_uint(q), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}


// acc = W·x, x = the state features vcat(θ,z)[axis_nn] (<= 16 of them).
// Compact fragments: [m][r < ks][lane] f32, k = 4r + lane_group.
// KS > 0: the chain-wide k-step count is a compile-time constant (FAST variant).
template <int HT, int TT, int KS = 0>
__device__ __forceinline__ void dense_first(const uint8_t* buf, const UNet& N, const float (&xin)[TT][4],
                                            f32x4 (&acc)[TT][HT]) {
    const int lane = threadIdx.x & 63;
    const float* wb = reinterpret_cast<const float*>(buf + N.off_w0) + lane;
    const int ks = KS > 0 ? KS : N.ks;
    if constexpr (KS > 0) {  // first k-step starts from an inline-zero accumulator
#pragma unroll
        for (int m = 0; m < HT; ++m) {
            const float w = wb[m * KS * 64];
#pragma unroll
            for (int t = 0; t < TT; ++t) acc[t][m] = mfma4(w, xin[t][0], f32x4{0.f, 0.f, 0.f, 0.f});
        }
#pragma unroll
        for (int r = 1; r < KS; ++r)
#pragma unroll
            for (int m = 0; m < HT; ++m) {
                const float w = wb[(m * KS + r) * 64];
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t][m] = mfma4(w, xin[t][r], acc[t][m]);
            }
        return;
    }
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int m = 0; m < HT; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (r < ks) {
#pragma unroll
            for (int m = 0; m < HT; ++m) {
                const float w = wb[(m * ks + r) * 64];
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t][m] = mfma4(w, xin[t][r], acc[t][m]);
            }
        }
    }
}

// out = W·in over a full H×H Dense (fragments [kq][m][lane][4] at wb).
// m-tiles are processed in pairs: two interleaved accumulator chains (64
// cycles apart >= the 40-cycle MFMA dependency latency) and only 2×2
// fragment registers in flight (next k-quad prefetched).
template <int HT, int TT>
__device__ __forceinline__ void dense_hidden(const uint8_t* wb, const f32x4 (&in)[TT][HT], f32x4 (&out)[TT][HT]) {
    const int lane = threadIdx.x & 63;
    wb += lane * 16;
    constexpr int MB = HT < 2 ? HT : 2;
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int m = 0; m < HT; ++m) out[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m0 = 0; m0 < HT; m0 += MB) {
        f32x4 w[2][MB];
#pragma unroll
        for (int mm = 0; mm < MB; ++mm) w[0][mm] = lds4(wb + (m0 + mm) * 1024);
#pragma unroll
        for (int kq = 0; kq < HT; ++kq) {
            const int cb = kq & 1;
            if (kq + 1 < HT) {
#pragma unroll
                for (int mm = 0; mm < MB; ++mm) w[cb ^ 1][mm] = lds4(wb + ((kq + 1) * HT + m0 + mm) * 1024);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int mm = 0; mm < MB; ++mm)
#pragma unroll
                    for (int t = 0; t < TT; ++t)
                        out[t][m0 + mm] = mfma4(w[cb][mm][r], in[t][kq][r], out[t][m0 + mm]);
        }
    }
}

// v = σ.(v .+ b)  — bias after the product (Flux: W*x .+ b).  add_bias false:
// the bias is already the last term of the MFMA chain (folded first Dense).
template <int HT, int TT, bool RELU>
__device__ __forceinline__ void bias_act(const uint8_t* bb, int act, f32x4 (&v)[TT][HT], bool add_bias = true) {
    const int g = (threadIdx.x & 63) >> 4;
    if (add_bias) {
#pragma unroll
        for (int m = 0; m < HT; ++m) {
            const f32x4 b = lds4(bb + ((16 * m + 4 * g) << 2));
#pragma unroll
            for (int t = 0; t < TT; ++t) v[t][m] = v[t][m] + b;
        }
    }
    if (RELU || act == DF_ACT_RELU) {
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int m = 0; m < HT; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[t][m][r] = relu_fast(v[t][m][r]);
    } else if (act != DF_ACT_IDENTITY) {
        if (!RELU) {
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int m = 0; m < HT; ++m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[t][m][r] = impl::act_fn(act, v[t][m][r]);
        }
    }
}

// Final Dense, <= 4 outputs, as a VALU GEMV; every lane ends with all outputs.
// NO > 0: the output count is a compile-time constant (FAST variant).
template <int HT, int TT, bool RELU, int NO = 0>
__device__ __forceinline__ void out_valu(const uint8_t* buf, const UNet& N, const f32x4 (&h)[TT][HT],
                                         f32x4 (&o)[TT]) {
    const int g = (threadIdx.x & 63) >> 4;
    const uint8_t* w3 = buf + N.off_out;
    constexpr int INP = 16 * HT;
    const int n_out = NO > 0 ? NO : N.n_out;
    const float* b3 = reinterpret_cast<const float*>(w3) + n_out * INP;
#pragma unroll
    for (int t = 0; t < TT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oo = 0; oo < 4; ++oo) {
        if (oo < n_out) {
            float p[TT];
#pragma unroll
            for (int t = 0; t < TT; ++t) p[t] = 0.f;
#pragma unroll
            for (int kq = 0; kq < HT; ++kq) {
                const f32x4 w = lds4(w3 + ((oo * INP + 16 * kq + 4 * g) << 2));
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int t = 0; t < TT; ++t) p[t] = __builtin_fmaf(w[r], h[t][kq][r], p[t]);
            }
            const float bo = b3[oo];
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const float v = xgroup_sum(p[t]) + bo;
                o[t][oo] = (RELU || N.act_out == DF_ACT_IDENTITY) ? v : impl::act_fn(N.act_out, v);
            }
        }
    }
}

// Final Dense, NO <= 4 outputs known at compile time (FAST variant), as a VALU
// GEMV whose lane-group reduction is a transpose: two v_permlane16_swap pair up
// outputs (0,1) and (2,3), one v_permlane32_swap completes them, so lane group g
// ends with output g — the transformed dim it updates — instead of every lane
// holding all outputs.  Sums associate as ((p0+p1)+(p2+p3)) over the groups,
// bitwise xgroup_sum's order; the bias is added after the product as in out_valu.
template <int HT, int TT, int NO>
__device__ __forceinline__ void out_valu_t(const uint8_t* buf, const UNet& N, const f32x4 (&h)[TT][HT],
                                           float (&y)[TT]) {
    static_assert(NO >= 1 && NO <= 4, "FAST tails: 1..4 outputs");
    const int g = (threadIdx.x & 63) >> 4;
    const uint8_t* w3 = buf + N.off_out;
    constexpr int INP = 16 * HT;
    float p[TT][4];
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int oo = 0; oo < 4; ++oo) p[t][oo] = 0.f;
#pragma unroll
    for (int oo = 0; oo < NO; ++oo)
#pragma unroll
        for (int kq = 0; kq < HT; ++kq) {
            const f32x4 w = lds4(w3 + ((oo * INP + 16 * kq + 4 * g) << 2));
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < TT; ++t) p[t][oo] = __builtin_fmaf(w[r], h[t][kq][r], p[t][oo]);
        }
    const float bo = reinterpret_cast<const float*>(w3)[NO * INP + (g < NO ? g : 0)];
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(p[t][0]), __float_as_uint(p[t][1]), false, false);
        const float A = __uint_as_float(a[0]) + __uint_as_float(a[1]);  // rows: p0 g01, p1 g01, p0 g23, p1 g23
        float Bv = 0.f;
        if constexpr (NO > 2) {
            auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(p[t][2]), __float_as_uint(p[t][3]), false, false);
            Bv = __uint_as_float(b[0]) + __uint_as_float(b[1]);             // p2 g01, p3 g01, p2 g23, p3 g23
        }
        auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(A), __float_as_uint(Bv), false, false);
        y[t] = (__uint_as_float(c[0]) + __uint_as_float(c[1])) + bo;      // group g: output g
    }
}

// Lane group 0 gets (y_0 + y_1) + ... + y_{NO-1} of the per-group outputs (row order, RNVP.jl:180).
template <int NO>
__device__ __forceinline__ float group_row_sum(float y) {
    float s = y;
    if constexpr (NO > 1) {  // group 1 → group 0
        auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(y), __float_as_uint(y), false, false);
        s = s + __uint_as_float(a[1]);
    }
    if constexpr (NO > 2) {  // groups 2, 3 → groups 0, 1
        auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false);
        const float y2 = __uint_as_float(b[1]);
        s = s + y2;
        if constexpr (NO > 3) {
            auto c = __builtin_amdgcn_permlane16_swap(__float_as_uint(y2), __float_as_uint(y2), false, false);
            s = s + __uint_as_float(c[1]);
        }
    }
    return s;
}

// Final Dense through MFMA (out <= 32): rows 16m + 4g + r in out[t][m].
template <int HT, int TT, bool RELU>
__device__ __forceinline__ void out_mfma(const uint8_t* buf, const UNet& N, const f32x4 (&h)[TT][HT],
                                         f32x4 (&out)[TT][2]) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const uint8_t* wb = buf + N.off_out + lane * 16;
    const int mt = (N.n_out + 15) >> 4;
#pragma unroll
    for (int t = 0; t < TT; ++t) out[t][0] = out[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kq = 0; kq < HT; ++kq) {
        const f32x4 w0 = lds4(wb + (kq * mt + 0) * 1024);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < TT; ++t) out[t][0] = mfma4(w0[r], h[t][kq][r], out[t][0]);
        if (mt > 1) {
            const f32x4 w1 = lds4(wb + (kq * mt + 1) * 1024);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < TT; ++t) out[t][1] = mfma4(w1[r], h[t][kq][r], out[t][1]);
        }
    }
    const uint8_t* bb = buf + N.off_out + HT * mt * 1024;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        if (m < mt) {
            const f32x4 b = lds4(bb + ((16 * m + 4 * g) << 2));
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                f32x4 v = out[t][m] + b;
                if (!RELU && N.act_out != DF_ACT_IDENTITY)
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = impl::act_fn(N.act_out, v[r]);
                out[t][m] = v;
            }
        }
    }
}

template <int PH>
__device__ __forceinline__ float couple1(float v, float y) {
    if (PH == impl::PH_S_FWD) return v * expf(y);
    if (PH == impl::PH_T_FWD) return v + y;
    if (PH == impl::PH_T_BWD) return v - y;
    return v * expf(-y);  // PH_S_BWD
}

// Output Dense + coupling phase of net N on the last hidden activations H.
// NO > 0: n_out = n_af = NO at compile time (FAST variant, OUTV only).
template <int HT, int TT, bool OUTV, bool RELU, int PH, int NO = 0>
__device__ __forceinline__ void tail(const uint8_t* buf, const UNet& N, const ULayer& L, const int32_t* tab,
                                     float* state, const int (&ro)[TT], float (&sum)[TT], const f32x4 (&H)[TT][HT]) {
    const int g = (threadIdx.x & 63) >> 4;
    constexpr bool SPH = (PH == impl::PH_S_FWD || PH == impl::PH_S_BWD);
    const int32_t* af = tab + L.af_tab;
    const int n_af = (OUTV && NO > 0) ? NO : L.n_af;
#pragma unroll
    for (int t = 0; t < TT; ++t) sum[t] = 0.f;
#ifdef DF_EXP_NOTAIL  // diagnostic build only: no output Dense / coupling (results are wrong)
    if (true) {
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            float acc = 0.f;
#pragma unroll
            for (int m = 0; m < HT; ++m) acc += H[t][m][0];
            asm volatile("" ::"v"(acc));
        }
        return;
    }
#endif
    if constexpr (OUTV && NO > 0) {
        float y[TT];
        out_valu_t<HT, TT, NO>(buf, N, H, y);
        const int slot = af[g < NO ? g : 0];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if (g < NO) state[ro[t] + slot] = couple1<PH>(state[ro[t] + slot], y[t]);
            if (SPH) sum[t] = group_row_sum<NO>(y[t]);  // valid in lane group 0 (ldj_update)
        }
    } else if constexpr (OUTV) {
        f32x4 o[TT];
        out_valu<HT, TT, RELU, NO>(buf, N, H, o);
        const int slot = (g < n_af) ? af[g] : 0;
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const float y = impl::sel4(o[t], g);
            if (g < n_af) state[ro[t] + slot] = couple1<PH>(state[ro[t] + slot], y);
            if (SPH) {
                // ldj = Σ_k s[k] in row order (RNVP.jl:180 / :86)
                float s_ = o[t][0];
#pragma unroll
                for (int oo = 1; oo < 4; ++oo)
                    if (oo < n_af) s_ = s_ + o[t][oo];
                sum[t] = s_;
            }
        }
    } else {
        f32x4 o[TT][2];
        out_mfma<HT, TT, RELU>(buf, N, H, o);
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            float p = 0.f;
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int oo = 16 * m + 4 * g + r;
                    if (oo < L.n_af) {
                        const int slot = af[oo];
                        const float y = o[t][m][r];
                        state[ro[t] + slot] = couple1<PH>(state[ro[t] + slot], y);
                        if (SPH) p = p + y;
                    }
                }
            if (SPH) sum[t] = xgroup_sum(p);
        }
    }
}

// ---- SPLIT variant: f32 GEMMs on bf16 MFMA (v_mfma_f32_16x16x32_bf16) ----
// Both operands are split in three bf16 planes, a = a0 + a1 + a2 exactly (RNE
// remainders, 8+8+8 significand bits; weights by the planner, activations here
// by v_cvt_pk_bf16_f32), and W·x is accumulated in f32 from the six products
// w0x0 + w0x1 + w1x0 + w0x2 + w1x1 + w2x0.  The dropped terms are below 2^-26
// of |w·x| and every product is exact, so the sums carry f32-level error
// (≈ Σ|w·x|·2^-24, like the exact-f32 MFMA chain) at 16/6 of its MFMA rate.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf(const bf16x8& a, const bf16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Remainder x - (float)h[S] of an RNE bf16 pair h, as one v_dot2c_f32_bf16
// (x + h·(-1, 0) or x + h·(0, -1)): the difference is exactly representable, and the
// dot2 returns it bitwise (tools/probe/dot2_split.hip), so the two bf16 → f32 unpacks
// and the f32 subtract of the plain form become one instruction per value.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#ifndef DF_SPLIT_DOT2
#define DF_SPLIT_DOT2 1
#endif
template <int S>
__device__ __forceinline__ float split_rem(bf16x2 h, float x) {
#if DF_SPLIT_DOT2 == 2
    // plain VALU: hi unpacked by a shift (low half) or a mask (high half), then one
    // v_sub_f32 (asm: -O3 would pair two of them into v_pk_add_f32).  Beside MFMAs a
    // v_dot2c_f32_bf16 or a packed f32 op waits for the matrix pipe (≈ 16 cycles each,
    // tools/probe/mfma_valu.hip); shifts, masks and subtracts co-issue.
    const uint32_t u = __builtin_bit_cast(uint32_t, h);
    const float hi = __uint_as_float(S == 0 ? (u << 16) : (u & 0xffff0000u));
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(hi));
    return r;
#elif DF_SPLIT_DOT2
    // (-1, 0) is materialised by a v_mov: the compiler would otherwise encode it as the
    // inline constant -1.0, which the hardware reads as the f32 0xbf800000, i.e. (0, -1)
    // (probe: tools/probe/dot2_split.hip).  The asm is pure, so it is hoisted and shared.
    uint32_t c;
    if (S == 0) asm("v_mov_b32 %0, 0xbf80" : "=v"(c));
    else c = 0xbf800000u;
    return __builtin_amdgcn_fdot2_f32_bf16(h, __builtin_bit_cast(bf16x2, c), x, false);
#else
    return x - (float)h[S];
#endif
}

// 2 f32 values → their three bf16 planes (pairs).
__device__ __forceinline__ void split2(float a, float b, bf16x2& p0, bf16x2& p1, bf16x2& p2) {
    p0 = bf16x2{(__bf16)a, (__bf16)b};
    const float ra = split_rem<0>(p0, a), rb = split_rem<1>(p0, b);
    p1 = bf16x2{(__bf16)ra, (__bf16)rb};
    p2 = bf16x2{(__bf16)split_rem<0>(p1, ra), (__bf16)split_rem<1>(p1, rb)};
}

// 8 f32 values → their three bf16 planes.
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
        bf16x2 h, m, l;
        split2(v[e], v[e + 1], h, m, l);
        p0[e] = h[0]; p0[e + 1] = h[1];
        p1[e] = m[0]; p1[e + 1] = m[1];
        p2[e] = l[0]; p2[e + 1] = l[1];
    }
}

// Remainders on the matrix pipe (DF_SPLIT_MREM): for one accumulator tile c (lane
// (g, j): rows 4g + r of sample j) and its RNE bf16 plane h (the same four values),
// v_mfma_f32_16x16x16_bf16 with A = −I and C = c gives c − h: the only non-zero
// product is −h, exact, and C + one product rounds once — to the exact difference
// (representable: h is c rounded to 8 significant bits).  Bitwise the dot2 remainder,
// one matrix instruction per 16 values instead of 16 v_dot2c_f32_bf16 (which cost
// ≈ 8–10 issue cycles each beside the MFMAs).  −I on the A operand: lane (g, i) holds
// A[i][4g + e], −1 iff 4g + e == i.  (A non-finite value of one row turns 0·inf into
// NaN for its whole sample — whose outputs are non-finite anyway.)
#ifndef DF_SPLIT_MREM
#define DF_SPLIT_MREM 1
#endif
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ short4v neg_eye() {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    short4v p;
#pragma unroll
    for (int e = 0; e < 4; ++e) p[e] = (4 * g + e == i) ? (short)0xbf80 : (short)0;
    return p;
}

__device__ __forceinline__ f32x4 mrem(short4v eye, bf16x4v h, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(eye, __builtin_bit_cast(short4v, h), c, 0, 0, 0);
}

// planes of two accumulator tiles (8 values: a then b), remainders on the matrix pipe
__device__ __forceinline__ void split8_mrem(short4v eye, const f32x4& a, const f32x4& b, bf16x8& p0, bf16x8& p1,
                                            bf16x8& p2) {
    bf16x4v h0, h1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        h0[e] = (__bf16)a[e];
        h1[e] = (__bf16)b[e];
    }
    p0 = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
    const f32x4 ra = mrem(eye, h0, a), rb = mrem(eye, h1, b);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        h0[e] = (__bf16)ra[e];
        h1[e] = (__bf16)rb[e];
    }
    p1 = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
    const f32x4 sa = mrem(eye, h0, ra), sb = mrem(eye, h1, rb);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        h0[e] = (__bf16)sa[e];
        h1[e] = (__bf16)sb[e];
    }
    p2 = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
}

// First Dense of a FAST net (one k-step, bias folded in slot g = 3): lane group g
// carries feature g's planes in the product slots (x0, x1, x0, x2, x1, x0, 0, 0)
// against the planner's (w0, w0, w1, w0, w1, w2, 0, 0): one MFMA per m-tile.
template <int HT, int TT>
__device__ __forceinline__ void dense_first_split(const uint8_t* buf, const UNet& N, const float (&xin)[TT][4],
                                                  f32x4 (&acc)[TT][HT]) {
    const int lane = threadIdx.x & 63;
    bf16x8 b[TT];
    const __bf16 z = (__bf16)0.f;
#pragma unroll
    for (int t = 0; t < TT; t += 2) {  // tiles in pairs: one split of two values
        bf16x2 h, m, l;
        split2(xin[t][0], t + 1 < TT ? xin[t + 1][0] : 0.f, h, m, l);
        b[t] = bf16x8{h[0], m[0], h[0], l[0], m[0], h[0], z, z};
        if (t + 1 < TT) b[t + 1] = bf16x8{h[1], m[1], h[1], l[1], m[1], h[1], z, z};
    }
    const uint8_t* wb = buf + N.off_w0 + lane * 16;
#pragma unroll
    for (int m = 0; m < HT; ++m) {
        const bf16x8 w = *reinterpret_cast<const bf16x8*>(wb + m * 1024);
#pragma unroll
        for (int t = 0; t < TT; ++t) acc[t][m] = mfma_bf(w, b[t], f32x4{0.f, 0.f, 0.f, 0.f});
    }
}

// Hidden H×H Dense: k-chunk c of 32 inputs = accumulator tiles 2c, 2c+1 (lane
// (g, j): rows 32c + 16(e>>2) + 4g + (e&3) of sample j), split on the fly.
// The accumulators start from the bias (b + W·x: the sum's rounding order differs
// from Flux's W*x .+ b by one f32 rounding, like any other summation order).
// BIAS false (the training kernel's W1ᵀδ): the chains start from zero.
template <int HT, int TT, bool BIAS = true, bool FENCE = false>
__device__ __forceinline__ void dense_hidden_split(const uint8_t* wb, const f32x4 (&in)[TT][HT],
                                                   f32x4 (&out)[TT][HT]) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const uint8_t* bb = wb + (HT / 2) * HT * 3072;
    wb += lane * 16;
    const short4v eye = DF_SPLIT_MREM ? neg_eye() : short4v{0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < HT; ++m) {
        const f32x4 b = BIAS ? lds4(bb + ((16 * m + 4 * g) << 2)) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < TT; ++t) out[t][m] = b;
    }
#pragma unroll
    for (int c = 0; c < HT / 2; ++c) {
        bf16x8 x[TT][3];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const float v[8] = {in[t][2 * c][0],     in[t][2 * c][1],     in[t][2 * c][2],     in[t][2 * c][3],
                                in[t][2 * c + 1][0], in[t][2 * c + 1][1], in[t][2 * c + 1][2], in[t][2 * c + 1][3]};
#ifdef DF_DIAG_NOSPLIT  // diagnostic build: hi plane only, repeated (results are wrong)
            for (int e = 0; e < 8; ++e) x[t][0][e] = (__bf16)v[e];
            x[t][1] = x[t][0];
            x[t][2] = x[t][0];
#else
            if constexpr (DF_SPLIT_MREM) split8_mrem(eye, in[t][2 * c], in[t][2 * c + 1], x[t][0], x[t][1], x[t][2]);
            else split8(v, x[t][0], x[t][1], x[t][2]);
#endif
        }
#pragma unroll
        for (int m = 0; m < HT; ++m) {
            const uint8_t* f = wb + (c * HT + m) * 3072;
            const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(f);
            const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(f + 1024);
            const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(f + 2048);
#pragma unroll
            for (int t = 0; t < TT; ++t) {  // small terms first
                f32x4 a = out[t][m];
                a = mfma_bf(w2, x[t][0], a);
                a = mfma_bf(w1, x[t][1], a);
                a = mfma_bf(w0, x[t][2], a);
                a = mfma_bf(w1, x[t][0], a);
                a = mfma_bf(w0, x[t][1], a);
                out[t][m] = mfma_bf(w0, x[t][0], a);
            }
            if (FENCE) asm volatile("" ::: "memory");  // fragment reads not hoisted past this m-tile
        }
    }
}

// Evaluate net N for TT 16-sample tiles (state rows ro[t]) and apply its
// coupling phase; sum[t] = Σ_k s_k for s phases (row order).
template <int HT, int TT, bool OUTV, bool RELU, int PH, bool FAST = false, int NO = 0, bool SPLIT = false>
__device__ __forceinline__ void net_tiles(const uint8_t* buf, const UNet& N, const ULayer& L, const int32_t* tab,
                                          float* state, const int (&ro)[TT], float (&sum)[TT]) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    constexpr bool SPH = (PH == impl::PH_S_FWD || PH == impl::PH_S_BWD);
    if constexpr (SPLIT && FAST && HT >= 2) {
        float xin[TT][4];
        const int slot = tab[L.feat_tab + g];
#pragma unroll
        for (int t = 0; t < TT; ++t) xin[t][0] = state[ro[t] + slot];
        f32x4 A[TT][HT], B[TT][HT];
        dense_first_split<HT, TT>(buf, N, xin, A);
        bias_act<HT, TT, true>(buf, DF_ACT_RELU, A, false);
        dense_hidden_split<HT, TT>(buf + N.off_h, A, B);
        bias_act<HT, TT, true>(buf, DF_ACT_RELU, B, false);
        tail<HT, TT, OUTV, RELU, PH, NO>(buf, N, L, tab, state, ro, sum, B);
        return;
    }
    // conditioner input: features k = 4r + g of vcat(θ,z)[axis_nn] (zero slot pads)
    float xin[TT][4];
    const int32_t* feat = tab + L.feat_tab;
    constexpr int KS = FAST ? 1 : 0;
    const int ks = FAST ? 1 : N.ks;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int slot = (r < ks) ? feat[4 * r + g] : 0;
#pragma unroll
        for (int t = 0; t < TT; ++t) xin[t][r] = (r < ks) ? state[ro[t] + slot] : 0.f;
    }

    f32x4 A[TT][HT], B[TT][HT];
    dense_first<HT, TT, KS>(buf, N, xin, A);
    bias_act<HT, TT, RELU>(buf + N.off_b0, N.act0, A, FAST ? false : !N.fold0);
    if (FAST || N.nh == 1) {  // the default _dflt_net (n_sublayers = 2): one H×H Dense
        dense_hidden<HT, TT>(buf + N.off_h, A, B);
        bias_act<HT, TT, RELU>(buf + N.off_h + HT * HT * 1024, N.acth, B);
        tail<HT, TT, OUTV, RELU, PH, NO>(buf, N, L, tab, state, ro, sum, B);
        return;
    }
    // hidden Denses alternate A -> B -> A ... (no register copies)
    bool in_a = true;
    for (int k = 0; k < N.nh; k += 2) {
        dense_hidden<HT, TT>(buf + N.off_h + k * N.hstride, A, B);
        bias_act<HT, TT, RELU>(buf + N.off_h + k * N.hstride + HT * HT * 1024, N.acth, B);
        in_a = false;
        if (k + 1 < N.nh) {
            dense_hidden<HT, TT>(buf + N.off_h + (k + 1) * N.hstride, B, A);
            bias_act<HT, TT, RELU>(buf + N.off_h + (k + 1) * N.hstride + HT * HT * 1024, N.acth, A);
            in_a = true;
        }
    }
    if (in_a) tail<HT, TT, OUTV, RELU, PH, NO>(buf, N, L, tab, state, ro, sum, A);
    else tail<HT, TT, OUTV, RELU, PH, NO>(buf, N, L, tab, state, ro, sum, B);
}

// The s-net and t-net of one RNVP layer evaluated together (FAST variant, exact f32,
// both nets in the resident stage, NO = n_af outputs each): they read the same
// conditioner features (vcat(θ,z)[axis_nn], RNVP.jl:174-177), so their MFMA chains and
// GEMV tails are independent and interleave, which halves the dependent latency of a
// layer for a wave that has no other work (small batches: profiles/r04_phase_cfg1.txt).
// The coupling is then applied in the reference's order with the same roundings as the
// two phases of net_tiles: forward z·exp(s) then + t (RNVP.jl:182-184), inverse (x − t)
// then ·exp(−s) (RNVP.jl:86-90); ssum[t] = Σ_k s_k in row order (lane group 0).
template <int HT, int TT, bool RELU, bool FWDP, int NO>
__device__ __forceinline__ void net_pair_tiles(const uint8_t* buf, const ULayer& L, const int32_t* tab, float* state,
                                               const int (&ro)[TT], float (&ssum)[TT]) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    float xin[TT][4];
    const int slot_in = tab[L.feat_tab + g];
#pragma unroll
    for (int t = 0; t < TT; ++t) xin[t][0] = state[ro[t] + slot_in];
    f32x4 As[TT][HT], At[TT][HT], Bs[TT][HT], Bt[TT][HT];
    dense_first<HT, TT, 1>(buf, L.s, xin, As);
    dense_first<HT, TT, 1>(buf, L.t, xin, At);
    bias_act<HT, TT, RELU>(buf + L.s.off_b0, L.s.act0, As, false);
    bias_act<HT, TT, RELU>(buf + L.t.off_b0, L.t.act0, At, false);
    dense_hidden<HT, TT>(buf + L.s.off_h, As, Bs);
    dense_hidden<HT, TT>(buf + L.t.off_h, At, Bt);
    bias_act<HT, TT, RELU>(buf + L.s.off_h + HT * HT * 1024, L.s.acth, Bs);
    bias_act<HT, TT, RELU>(buf + L.t.off_h + HT * HT * 1024, L.t.acth, Bt);
    float ys[TT], yt[TT];
    out_valu_t<HT, TT, NO>(buf, L.s, Bs, ys);
    out_valu_t<HT, TT, NO>(buf, L.t, Bt, yt);
    const int slot = tab[L.af_tab + (g < NO ? g : 0)];
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        if (g < NO) {
            float v = state[ro[t] + slot];
            if (FWDP) {
                v = v * expf(ys[t]);
                v = v + yt[t];
            } else {
                v = v - yt[t];
                v = v * expf(-ys[t]);
            }
            state[ro[t] + slot] = v;
        }
        ssum[t] = group_row_sum<NO>(ys[t]);
    }
}

}  // namespace uni

#ifndef DF_UNI_WAVES
#define DF_UNI_WAVES 4
#endif
#ifndef DF_FAST_WAVES
#define DF_FAST_WAVES 4
#endif

template <int HT, int MODE, bool OUTV, bool RELU, bool FAST = false, bool SPLIT = false>
__global__ void __launch_bounds__(kBlockThreads, FAST ? DF_FAST_WAVES : DF_UNI_WAVES)
uniform_kernel(ChainArgs a) {
    using namespace uni;
    constexpr bool FWD = (MODE == MODE_FWD || MODE == MODE_FWD_INPLACE);
    constexpr bool WANT_LDJ = (MODE != MODE_FWD_INPLACE);

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int stage_area = a.stage_bytes * a.n_stage_bufs;
    int32_t* tab = reinterpret_cast<int32_t*>(smem + stage_area);
    float* state = reinterpret_cast<float*>(smem + stage_area + a.tab_bytes);

    ClockStamp clk;
    clk.begin(a);
#ifdef DF_PHASE_STAMPS  // diagnostic build (wrong outputs): wave 0 of workgroup 0 stamps its phases
    uint64_t ph[16] = {};
#define DF_PH(i) do { if (blockIdx.x == 0 && threadIdx.x == 0) ph[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define DF_PH(i) do {} while (0)
#endif
    DF_PH(0);
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int d = a.d, n = a.n, stride = a.stride, nd = n + d;
    const int nt = a.tiles;
    const int S = kWavesPerBlock * 16 * nt;
    const int cA = nd + 1, cE = nd + 2;
    const int64_t s0 = (int64_t)blockIdx.x * S;
    const int nvalid = (int)((a.batch - s0) < S ? (a.batch - s0) : S);

    Stager sg;
    sg.base = smem;
    sg.bytes = a.stage_bytes;
    sg.sched = FWD ? a.sched_fwd : a.sched_bwd;
    sg.n = FWD ? a.n_sched_fwd : a.n_sched_bwd;
    impl::stager_start(sg, a);

    // Copy-in of the tables, the NormalizationLayer bounds (a.params, kept in LDS right
    // after the tables) and the state tile.  Fast form: every thread issues ALL its loads
    // — up to four table words, one bound, one θ bound per lane, its sample row's z and
    // θ — before its first LDS store, so the copy costs one memory latency; three serial
    // load → store loops cost three (≈1.5 k cycles each, profiles/r04_phase_cfg1.txt),
    // which is a third of a config-1 launch at B = 4096.
    float* tabf = reinterpret_cast<float*>(tab);
    constexpr int kRowMax = 8;  // fast copy-in: d, n <= 8 (every default-shape chain of the configs)
    const bool fast_copy = d <= kRowMax && n <= kRowMax && a.n_par <= kBlockThreads && a.tab_ints <= 4 * kBlockThreads;
    auto row_init = [&](int smp) {  // [0 | ldj_chain | ldj_elem | 1 (folded-bias input)]
        for (int c = nd; c < stride; ++c) state[smp * stride + c] = (c == nd + 3) ? 1.f : 0.f;
    };
    auto theta_in = [&](float v, float lo, float hi) {  // normalize_input (Data.jl:213-218)
        const float diff = hi - lo;
        return (diff == 0.f) ? 0.f : (v - lo) / diff;
    };
    if (fast_copy) {
        const int n_tab = a.tab_ints, n_par = a.n_par;
        int tv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + u * kBlockThreads;
            tv[u] = i < n_tab ? a.tables[i] : 0;
        }
        const float pv = tid < n_par ? a.params[tid] : 0.f;
        const bool norm_th = a.tmin != nullptr;
        const float blo = (norm_th && lane < n) ? a.tmin[lane] : 0.f;  // lane c: column c's bounds
        const float bhi = (norm_th && lane < n) ? a.tmax[lane] : 0.f;
        const int smp = tid;                                           // this thread's first row
        const bool valid = smp < nvalid;
        float zr[kRowMax], tr[kRowMax];
#pragma unroll
        for (int c = 0; c < kRowMax; ++c)
            if (c < d) zr[c] = valid ? a.zin[(s0 + smp) * d + c] : 0.f;
#pragma unroll
        for (int c = 0; c < kRowMax; ++c)
            if (c < n) tr[c] = valid ? a.theta[(s0 + smp) * n + c] : 0.f;
        // every load is in flight: the stores
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + u * kBlockThreads;
            if (i < n_tab) tab[i] = tv[u];
        }
        if (tid < n_par) tabf[n_tab + tid] = pv;
#pragma unroll
        for (int c = 0; c < kRowMax; ++c)
            if (c < n) {
                const float lo = __shfl(blo, c), hi = __shfl(bhi, c);
                if (smp < S) state[smp * stride + c] = (norm_th && valid) ? theta_in(tr[c], lo, hi) : tr[c];
            }
        if (smp < S) {
#pragma unroll
            for (int c = 0; c < kRowMax; ++c)
                if (c < d) state[smp * stride + n + c] = zr[c];
            row_init(smp);
        }
        // rows beyond the first kBlockThreads (tiles > 4): element by element
        for (int i = tid + kBlockThreads * d; i < S * d; i += kBlockThreads) {
            const int r = i / d, c = i - r * d;
            state[r * stride + n + c] = r < nvalid ? a.zin[(s0 + r) * d + c] : 0.f;
        }
        for (int i = tid + kBlockThreads * n; i < S * n; i += kBlockThreads) {
            const int r = i / n, c = i - r * n;
            float v = 0.f;
            if (r < nvalid) {
                v = a.theta[(s0 + r) * n + c];
                if (norm_th) v = theta_in(v, a.tmin[c], a.tmax[c]);
            }
            state[r * stride + c] = v;
        }
        for (int r = tid + kBlockThreads; r < S; r += kBlockThreads) row_init(r);
    } else {
        for (int i = tid; i < a.tab_ints; i += kBlockThreads) tab[i] = a.tables[i];
        for (int i = tid; i < S * d; i += kBlockThreads) {
            const int smp = i / d, c = i - smp * d;
            float v = 0.f;
            if (smp < nvalid) v = a.zin[(s0 + smp) * d + c];
            state[smp * stride + n + c] = v;
        }
        for (int i = tid; i < S * n; i += kBlockThreads) {
            const int smp = i / n, c = i - smp * n;
            float v = 0.f;
            if (smp < nvalid) {
                v = a.theta[(s0 + smp) * n + c];
                if (a.tmin) v = theta_in(v, a.tmin[c], a.tmax[c]);
            }
            state[smp * stride + c] = v;
        }
        for (int i = tid; i < S; i += kBlockThreads) row_init(i);
    }
    DF_PH(1);
    DF_PH(2);
    DF_PH(3);
    __syncthreads();
    DF_PH(4);

    const int row0 = ((wave * nt) * 16 + j) * stride;  // tile tt: row0 + tt*16*stride
#ifdef DF_NO_PAIR  // A/B build: the s and t nets of a layer one after the other
    constexpr bool no_pair = true;
#else
    constexpr bool no_pair = false;
#endif
    const int tstep = 16 * stride;
    bool have_acc = false;

    auto ldj_update = [&](int ro, float l, bool first_in_elem, bool last_in_elem) {
        if (!WANT_LDJ || g != 0) return;
        const float e = first_in_elem ? l : state[ro + cE] + l;
        state[ro + cE] = e;
        if (last_in_elem) state[ro + cA] = have_acc ? state[ro + cA] + e : e;
    };

    for (int it = 0; it < a.n_layers; ++it) {
        const int li = FWD ? it : a.n_layers - 1 - it;
        // descriptors through the constant address space: scalar loads (the host
        // writes them before the launch; nothing in the kernel stores to them)
        using CULayer = const __attribute__((address_space(4))) ULayer;
#ifdef DF_PHASE_STAMPS  // diagnostic: the whole descriptor loaded (and waited for) up front
        const ULayer L = *(const ULayer*)(&((CULayer*)(uintptr_t)a.ulayers)[li]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (it == 1) DF_PH(13);
#else
        const ULayer& L = *(const ULayer*)(&((CULayer*)(uintptr_t)a.ulayers)[li]);
#endif
        const int kind = L.kind;
        const bool first_in_elem = FWD ? L.elem_start : L.elem_end;
        const bool last_in_elem = FWD ? L.elem_end : L.elem_start;
        if (kind == DF_LAYER_NORM) {
            const float al = L.alpha, be = L.beta, delta = be - al;
            auto norm = [&](const auto* xmn) {
                const auto* xmx = xmn + d;
                for (int tt = 0; tt < nt; ++tt) {
                    const int ro = row0 + tt * tstep;
                    for (int i = g; i < d; i += 4) {
                        const float lo = xmn[i], hi = xmx[i], xd = hi - lo;
                        float v = state[ro + n + i];
                        if (FWD) v = ((xd * v - al * hi) + be * lo) / delta;
                        else v = (be * (v - lo) + al * (hi - v)) / xd;
                        state[ro + n + i] = v;
                    }
                    ldj_update(ro, FWD ? L.ldj_const : -L.ldj_const, first_in_elem, last_in_elem);
                }
            };
            if (fast_copy) norm(tabf + a.tab_ints + L.norm_off);  // the bounds were copied to LDS
            else norm(a.params + L.norm_off);
        } else {
            const bool rnvp = (kind == DF_LAYER_RNVP);
            // this wave's tiles in groups of kTT (nt is a multiple of kTT)
            constexpr int kTT = FAST ? kFastTileGroup : kUniformTileGroup;
            auto tiles_loop = [&](const UNet& N, auto ph_tag, auto no_tag, bool sphase, float sign) {
                constexpr int PH = decltype(ph_tag)::value;
                constexpr int NO = decltype(no_tag)::value;
                const uint8_t* buf = sg.buf();
                for (int tt = 0; tt < nt; tt += kTT) {
                    int ro[kTT];
                    float ssum[kTT];
                    // SPLIT: the row offsets from one opaque copy of row0 per tile group:
                    // left to itself the compiler strength-reduces every state address of
                    // the loop into its own VGPR induction variable (six), which the SPLIT
                    // kernel at 128 VGPRs spills — and a reload's vmcnt(0) also waits for the
                    // stage DMA issued just before (headline 1583 -> 1623 Msamples/s,
                    // gpurun_out/ab4e; the exact-f32 kernels keep the induction variables:
                    // config 1 at 2^20 lost 0.9% with the opaque copy)
                    int r0 = row0;
                    if constexpr (SPLIT) asm volatile("" : "+v"(r0));
#pragma unroll
                    for (int t = 0; t < kTT; ++t) ro[t] = r0 + (tt + t) * tstep;
                    net_tiles<HT, kTT, OUTV, RELU, PH, FAST, NO, SPLIT>(buf, N, L, tab, state, ro, ssum);
#pragma unroll
                    for (int t = 0; t < kTT; ++t) {
                        if (sphase) ldj_update(ro[t], sign * ssum[t], first_in_elem, last_in_elem);
                        else if (!rnvp) ldj_update(ro[t], 0.f, first_in_elem, last_in_elem);
                    }
                }
            };
            auto run_net = [&](const UNet& N, auto ph_tag, bool sphase, float sign) {
                impl::ensure_stage(N.stage, sg, a);
                if constexpr (FAST && OUTV) {  // output count fixed per net: branch-free tails
                    switch (N.n_out) {
                        case 1: tiles_loop(N, ph_tag, std::integral_constant<int, 1>{}, sphase, sign); break;
                        case 2: tiles_loop(N, ph_tag, std::integral_constant<int, 2>{}, sphase, sign); break;
                        case 3: tiles_loop(N, ph_tag, std::integral_constant<int, 3>{}, sphase, sign); break;
                        default: tiles_loop(N, ph_tag, std::integral_constant<int, 4>{}, sphase, sign); break;
                    }
                } else {
                    tiles_loop(N, ph_tag, std::integral_constant<int, 0>{}, sphase, sign);
                }
            };
            using PSF = std::integral_constant<int, impl::PH_S_FWD>;
            using PTF = std::integral_constant<int, impl::PH_T_FWD>;
            using PTB = std::integral_constant<int, impl::PH_T_BWD>;
            using PSB = std::integral_constant<int, impl::PH_S_BWD>;
            bool paired = false;
            if constexpr (FAST && OUTV && !SPLIT && HT <= 2) {
                // s and t together when both sit in one stage with the same output count
                if (rnvp && L.s.stage == L.t.stage && L.s.n_out == L.t.n_out && !no_pair) {
                    impl::ensure_stage(L.s.stage, sg, a);
                    auto pair_loop = [&](auto no_tag) {
                        constexpr int NO = decltype(no_tag)::value;
                        const uint8_t* buf = sg.buf();
                        for (int tt = 0; tt < nt; tt += kTT) {
                            int ro[kTT];
                            float ssum[kTT];
#pragma unroll
                            for (int t = 0; t < kTT; ++t) ro[t] = row0 + (tt + t) * tstep;
                            net_pair_tiles<HT, kTT, RELU, FWD, NO>(buf, L, tab, state, ro, ssum);
#pragma unroll
                            for (int t = 0; t < kTT; ++t)
                                ldj_update(ro[t], FWD ? ssum[t] : -ssum[t], first_in_elem, last_in_elem);
                        }
                    };
                    switch (L.s.n_out) {
                        case 1: pair_loop(std::integral_constant<int, 1>{}); break;
                        case 2: pair_loop(std::integral_constant<int, 2>{}); break;
                        case 3: pair_loop(std::integral_constant<int, 3>{}); break;
                        default: pair_loop(std::integral_constant<int, 4>{}); break;
                    }
                    paired = true;
                }
            }
            if (paired) {
            } else if (FWD) {
#ifdef DF_PHASE_STAMPS
                if (it == 1) DF_PH(11);
#endif
                if (rnvp) run_net(L.s, PSF{}, true, 1.f);
#ifdef DF_PHASE_STAMPS
                if (it == 1) DF_PH(12);
#endif
                run_net(L.t, PTF{}, false, 1.f);
            } else {
                run_net(L.t, PTB{}, false, 1.f);
                if (rnvp) run_net(L.s, PSB{}, true, -1.f);  // ln_det_jac = -Σ s
            }
        }
        have_acc = have_acc || last_in_elem;
#ifdef DF_PHASE_STAMPS
        if (it == 0) DF_PH(5);
        if (it == 1) DF_PH(6);
        if (it == 2) DF_PH(7);
        if (it == 3) DF_PH(8);
#endif
        if (!FWD && a.snap) {  // training: keep every layer's output for the reverse sweep
            float* dst = a.snap + (int64_t)li * a.batch * d;
            for (int tt = 0; tt < nt; ++tt) {
                const int smp = (wave * nt + tt) * 16 + j;
                if (smp < nvalid)
                    for (int i = g; i < d; i += 4) dst[(s0 + smp) * d + i] = state[row0 + tt * tstep + n + i];
            }
        }
    }

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (MODE == MODE_LOGPDF) {
        double part = 0.0;
        if (g == 0) {
            for (int tt = 0; tt < nt; ++tt) {
                const int ro = row0 + tt * tstep;
                const int smp = (wave * nt + tt) * 16 + j;
                float q = 0.f;
                for (int i = 0; i < d; ++i) {
                    const float zz = state[ro + n + i];
                    q = q + zz * zz;
                }
                const float lp = (a.c0 - q / 2.f) + state[ro + cA];
                if (smp < nvalid) {
                    if (a.lp_out) a.lp_out[s0 + smp] = lp;
                    part += (double)lp;
                }
            }
        }
        if (a.partial) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
            __syncthreads();
            double* red = reinterpret_cast<double*>(smem);
            if (lane == 0) red[wave] = part;
            __syncthreads();
            if (tid == 0) {
                double s = 0.0;
                for (int w = 0; w < kWavesPerBlock; ++w) s += red[w];
                a.partial[blockIdx.x] = s;
            }
        }
        if (!a.xout) {
            clk.end(a);
            return;
        }
    }
    __syncthreads();
    for (int i = tid; i < S * d; i += kBlockThreads) {
        const int smp = i / d, c = i - smp * d;
        if (smp < nvalid) a.xout[(s0 + smp) * d + c] = state[smp * stride + n + c];
    }
    if (WANT_LDJ && MODE != MODE_LOGPDF && a.ldj_out) {
        for (int i = tid; i < nvalid; i += kBlockThreads) a.ldj_out[s0 + i] = state[i * stride + cA];
    }
    DF_PH(9);
#ifdef DF_PHASE_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DF_PH(10);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < 14; ++i) a.xout[i] = (float)(ph[i] - ph[0]);
    }
#endif
#undef DF_PH
    clk.end(a);
}

template <int HT, bool RELU, bool FAST = false, bool SPLIT = false>
void* uniform_kernel_ptr_r(int mode, bool outv) {
#define DF_U(M) (outv ? reinterpret_cast<void*>(&uniform_kernel<HT, M, true, RELU, FAST, SPLIT>) \
                      : reinterpret_cast<void*>(&uniform_kernel<HT, M, false, RELU, FAST, SPLIT>))
    switch (mode) {
        case MODE_FWD: return DF_U(MODE_FWD);
        case MODE_FWD_INPLACE: return DF_U(MODE_FWD_INPLACE);
        case MODE_BWD: return DF_U(MODE_BWD);
        default: return DF_U(MODE_LOGPDF);
    }
#undef DF_U
}

// variant index: bit 0 = OUTV, bit 1 = RELU, bit 2 = FAST (RELU only: one first-Dense
// k-step with the bias folded in, chain-wide), bit 3 = SPLIT (FAST with OUTV on the
// bf16x3 split stages; hidden widths 32 and 64)
template <int HT>
void* uniform_kernel_ptr(int mode, int variant) {
    const bool outv = variant & 1;
    if constexpr (HT >= 2) {
        if ((variant & 8) && (variant & 4) && outv) return uniform_kernel_ptr_r<HT, true, true, true>(mode, true);
    }
    if (variant & 8) return nullptr;
    if (variant & 4) return uniform_kernel_ptr_r<HT, true, true>(mode, outv);
    return (variant & 2) ? uniform_kernel_ptr_r<HT, true>(mode, outv) : uniform_kernel_ptr_r<HT, false>(mode, outv);
}

template <int HT>
hipError_t launch_uniform_ht(int mode, int variant, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st) {
    void* args[] = {const_cast<ChainArgs*>(&a)};
    return hipLaunchKernel(uniform_kernel_ptr<HT>(mode, variant), dim3(grid), dim3(kBlockThreads), args, lds, st);
}

template <int HT>
hipError_t set_uniform_lds_limit_ht(size_t lds) {
    for (int mode = 0; mode < 4; ++mode)
        for (int v = 0; v < 16; ++v) {
            void* k = uniform_kernel_ptr<HT>(mode, v);
            if (!k) continue;
            hipError_t e = hipFuncSetAttribute(k,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

template <int HT>
hipError_t uniform_occupancy_ht(int mode, int variant, size_t lds, int* blocks) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, uniform_kernel_ptr<HT>(mode, variant), kBlockThreads,
                                                        lds);
}

}  // namespace df
