// df_chain_impl.h — fused CDNA4 (gfx950) kernel for the DensityFlows.jl
// FlowChain hot path: forward / backward (inverse) / forward! / logpdf.
// Included once per kernel variant (DF_HT) by df_kernels_ht*.hip.
//
// One workgroup (8 waves) owns S = 8·16·T consecutive samples.  Their state
// rows [θ | z | 0] live in LDS for the whole chain; each wave owns 16·T rows.
// Per coupling layer (src/affine/RNVP.jl:168-205, NICE.jl:118-170):
//   * the conditioner input vcat(θ,z)[axis_nn] is gathered from LDS through a
//     per-layer slot table (bit-exact index selection);
//   * every Dense of the s and t nets runs on v_mfma_f32_16x16x4_f32 with the
//     samples as the MFMA column dimension: A = weight fragments read from the
//     LDS stage buffer (packed by df_plan.cpp), B = activations held in
//     registers.  An accumulator tile is directly the B operand of the next
//     Dense (k = 16·tile + 4·lane_group + reg), so activations never leave
//     registers;
//   * bias (W*x .+ b, added after the product as Flux does) and σ are applied
//     to the accumulators; a final Dense with <= 4 outputs is a VALU GEMV;
//   * the coupling x_af = z_af·exp(s) + t is applied in two in-place phases,
//     one right after each net: forward  z·exp(s) (s-net) then + t (t-net);
//     inverse (x - t) (t-net) then ·exp(-s) (s-net).  Julia rounds the
//     product and the sum separately, so the phases are bit-identical to the
//     fused expression, and the conditioner input never contains transformed
//     dims (planner check), so the second net sees the same input;
//   * ldj = ±Σ s is accumulated per FlowElement and chain exactly as the
//     reference groups it (Blocks.jl:136,149, Chains.jl:160,179).
// Weights are staged global→LDS in stages (several layers per stage when they
// fit); the stage cache is uniform across the workgroup.
//
// Compiled with -ffp-contract=off: element-wise arithmetic is rounded op by
// op as Julia does (no implicit FMA); the MFMA products are exact f32 FMA
// chains.
#pragma once

#include <hip/hip_runtime.h>

#include "df_kernels.h"

namespace df {

typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef DF_WAVES_PER_EU
#define DF_WAVES_PER_EU(HT) ((HT) <= 4 ? 4 : 2)
#endif

namespace impl {

// relu = max(0, x) as ONE v_max_i32 on the bit pattern: non-negative floats order
// like their integer images, negatives and -0 map to +0, and NaNs with the sign
// bit clear (every NaN the GPU produces) propagate as in Julia.
__device__ __forceinline__ float relu(float x) {
    return __int_as_float(__builtin_elementwise_max(__float_as_int(x), 0));
}

// Flux 0.16's Dense evaluates σ = NNlib.fast_act(σ, x): tanh → tanh_fast,
// sigmoid → sigmoid_fast (Float32 methods, NNlib src/activations.jl).
// tanh_fast: x·n(x²)/d(x²), evalpoly's muladd Horner chains (fused), sign(x)
// once x² >= 66 (NaN stays NaN, as Julia's sign).
__device__ __forceinline__ float tanh_fast(float x) {
    const float x2 = x * x;
    const float n = fmaf(fmaf(fmaf(fmaf(1.587199e-8f, x2, 2.2332108e-5f), x2, 0.0035974074f), x2, 0.1346604f), x2, 1.0f);
    const float d =
        fmaf(fmaf(fmaf(fmaf(8.7767893e-7f, x2, 0.0003453992f), x2, 0.026262015f), x2, 0.4679937f), x2, 1.0f);
    return (x2 < 66.f) ? x * (n / d) : (x > 0.f ? 1.f : (x < 0.f ? -1.f : x));
}

// sigmoid_fast: NNlib.sigmoid with the saturations x > 40 → 1, x < -80 → 0.
__device__ __forceinline__ float sigmoid_fast(float x) {
    const float t = expf(-fabsf(x));
    const float y = (x >= 0.f) ? 1.f / (1.f + t) : t / (1.f + t);
    return (x > 40.f) ? 1.f : ((x < -80.f) ? 0.f : y);
}

__device__ __noinline__ float act_fn(int act, float x) {
    switch (act) {
        case DF_ACT_IDENTITY: return x;
        case DF_ACT_RELU: return relu(x);  // max(0, x), NaN-propagating
        case DF_ACT_TANH: return tanh_fast(x);
        case DF_ACT_SIGMOID: return sigmoid_fast(x);
        case DF_ACT_SOFTPLUS: return log1pf(expf(-fabsf(x))) + ((x > 0.f) ? x : 0.f);
        case DF_ACT_LOGCOSH: {  // x + softplus(-2x) - log(2)
            float y = -2.f * x;
            float sp = log1pf(expf(-fabsf(y))) + ((y > 0.f) ? y : 0.f);
            return (x + sp) - 0.6931471805599453f;
        }
        case DF_ACT_LEAKYRELU: return (x > 0.f) ? x : 0.01f * x;
        case DF_ACT_ELU: return (x > 0.f) ? x : expm1f(x);
        case DF_ACT_SWISH: {
            float t = expf(-fabsf(x));
            float sg = (x >= 0.f) ? 1.f / (1.f + t) : t / (1.f + t);
            return x * sg;
        }
        default: return x;
    }
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 lds4(const uint8_t* p) { return *reinterpret_cast<const f32x4*>(p); }

struct Smem {
    const int32_t* tab;
    float* state;
};

// Weight staging: stages are copied global -> LDS by DMA (global_load_lds,
// 16 B per lane, 1 KiB per wave instruction) into two LDS buffers.  The host
// computed the order in which this pass needs its stages (sched); while stage
// sched[i] is being consumed from buffer i&1, stage sched[i+1] is already in
// flight into the other buffer.  One workgroup barrier per stage switch.
struct Stager {
    uint8_t* base;        // LDS buffer 0; buffer 1 at base + bytes
    int bytes;            // per-buffer size
    const int32_t* sched; // stage schedule of this pass
    int n;                // schedule length
    int idx;              // schedule position of the resident stage
    int cur;              // resident stage id
    __device__ __forceinline__ uint8_t* buf() const { return base + ((idx & 1) ? bytes : 0); }
};

// Stage descriptors and schedules are read through the constant address space (scalar
// loads: the host writes them before the launch, nothing in a kernel stores to them) and
// the wave index is made scalar: read as generic pointers they were vector loads, each
// followed by a vmcnt(0) wait, and the source address a VGPR pair (spilled in the
// FAST SPLIT kernel, whose reload's vmcnt(0) then also waited for the DMA just issued).
template <typename T>
__device__ __forceinline__ T cload(const T* p, int64_t i) {
    using CT = const __attribute__((address_space(4))) T;
    return *(const T*)(&((CT*)(uintptr_t)p)[i]);
}

__device__ __forceinline__ void dma_stage(const ChainArgs& a, int s, uint8_t* dst) {
    const DevStage st = cload(a.stages, s);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint8_t* src = a.blob + st.src_off;
    const int nchunk = st.bytes >> 10;
    for (int c = wave; c < nchunk; c += kWavesPerBlock) {
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (c << 10) + lane * 16),
                                         (__attribute__((address_space(3))) void*)(dst + (c << 10)),
                                         16, 0, 0);
    }
}

__device__ __forceinline__ void stager_start(Stager& sg, const ChainArgs& a) {
    sg.idx = -1;
    sg.cur = -1;
    if (sg.n > 0) dma_stage(a, cload(sg.sched, 0), sg.base);
}

// Make stage `s` resident (uniform across the workgroup).
__device__ __forceinline__ void ensure_stage(int s, Stager& sg, const ChainArgs& a) {
    if (s == sg.cur) return;
#ifdef DF_EXP_NOSYNC  // diagnostic build only: no stage switches (results are wrong)
    if (sg.cur >= 0) { sg.cur = s; return; }
#endif
    const int nidx = sg.idx + 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA for sched[nidx] landed
    __syncthreads();                                     // ... every wave's, and buffer (nidx+1)&1 is free
    sg.idx = nidx;
    sg.cur = s;
    if (nidx >= sg.n || cload(sg.sched, nidx) != s) {
        // off-schedule request (not produced by the planner): synchronous copy
        const DevStage st = cload(a.stages, s);
        const f32x4* src = reinterpret_cast<const f32x4*>(a.blob + st.src_off);
        f32x4* dst = reinterpret_cast<f32x4*>(sg.buf());
        for (int i = threadIdx.x; i < (st.bytes >> 4); i += kBlockThreads) dst[i] = src[i];
        __syncthreads();
        sg.n = 0;  // schedule abandoned: every further switch copies synchronously
        return;
    }
    if (nidx + 1 < sg.n) dma_stage(a, cload(sg.sched, nidx + 1), sg.base + (((nidx + 1) & 1) ? sg.bytes : 0));
}

constexpr int out_tiles(int HT) { return HT < 2 ? HT : 2; }

template <int HT, int T, bool OUTV>
struct NetRegs {
    f32x4 h[T][HT];    // activations of the previous Dense (B operands)
    f32x4 acc[T][HT];  // accumulators of the current Dense
    // net output: OUTV: out[tt][0] = (o0..o3) in every lane group;
    // MFMA path: out[tt][m] = rows 16m + 4g + r
    f32x4 out[T][OUTV ? 1 : out_tiles(HT)];
};

// One MFMA Dense: acc = W · input (+ b, σ).  IN_STATE gathers the input
// features of vcat(θ,z)[axis_nn] from the LDS state rows.
template <int HT, int T>
__device__ __forceinline__ void dense_mfma(const ChainArgs& a, const DevDense& D, const int32_t* feat,
                                           Stager& sg, const Smem& sm, const int (&rowoff)[T],
                                           f32x4 (&h)[T][HT], f32x4 (&acc)[T][HT]) {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    constexpr int MG = (T == 1) ? 2 : 1;  // m-tiles per A-fragment group (independent MFMA chains)
#pragma unroll
    for (int tt = 0; tt < T; ++tt)
#pragma unroll
        for (int m = 0; m < HT; ++m) acc[tt][m] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c = 0; c < D.n_chunks; ++c) {
        const DevChunk C = a.chunks[D.chunk0 + c];
        ensure_stage(C.stage, sg, a);
        const uint8_t* base = sg.buf() + C.lds_off + lane * 16;
        if (D.in_kind == IN_STATE) {
#pragma unroll
            for (int kq = 0; kq < kMaxState / 16; ++kq) {
                if (kq >= C.kq_begin && kq < C.kq_end) {
                    float xin[T][4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int s = 4 * kq + r;
                        if (s < D.ks) {
                            const int slot = feat[4 * s + g];
#pragma unroll
                            for (int tt = 0; tt < T; ++tt) xin[tt][r] = sm.state[rowoff[tt] + slot];
                        } else {
#pragma unroll
                            for (int tt = 0; tt < T; ++tt) xin[tt][r] = 0.f;
                        }
                    }
                    const uint8_t* bq = base + (kq - C.kq_begin) * D.mt * 1024;
                    if (HT >= 8 && D.mt == HT) {
                        // full-M first Dense of a wide net: no per-tile guards, 4 chains
                        constexpr int MB = HT < 4 ? HT : 4;
                        const int rmax = D.ks - 4 * kq;  // k-steps of this k-quad that carry features
#pragma unroll
                        for (int m0 = 0; m0 < HT; m0 += MB) {
                            f32x4 w[MB];
#pragma unroll
                            for (int mm = 0; mm < MB; ++mm) w[mm] = lds4(bq + (m0 + mm) * 1024);
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (r < rmax)
#pragma unroll
                                    for (int mm = 0; mm < MB; ++mm)
#pragma unroll
                                        for (int tt = 0; tt < T; ++tt)
                                            acc[tt][m0 + mm] = mfma4(w[mm][r], xin[tt][r], acc[tt][m0 + mm]);
                        }
                        continue;
                    }
#pragma unroll
                    for (int m0 = 0; m0 < HT; m0 += MG) {
                        if (m0 < D.mt) {
                            f32x4 w[MG];
#pragma unroll
                            for (int mm = 0; mm < MG; ++mm)
                                w[mm] = (m0 + mm < D.mt) ? lds4(bq + (m0 + mm) * 1024) : f32x4{0, 0, 0, 0};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                if (4 * kq + r < D.ks) {
#pragma unroll
                                    for (int mm = 0; mm < MG; ++mm)
                                        if (m0 + mm < HT && m0 + mm < D.mt)
#pragma unroll
                                            for (int tt = 0; tt < T; ++tt)
                                                acc[tt][m0 + mm] = mfma4(w[mm][r], xin[tt][r], acc[tt][m0 + mm]);
                                }
                            }
                        }
                    }
                }
            }
        } else if (D.mt == HT && C.kq_begin == 0 && C.kq_end == HT) {
            // full-width hidden Dense in one stage: guard-free, fully unrolled.
            // MB independent accumulators interleaved per k-step (no MFMA
            // dependency stalls); the next k-quad's fragments are read from LDS
            // while the current one's MFMAs issue.
            constexpr int MB = HT < 4 ? HT : 4;
#pragma unroll
            for (int m0 = 0; m0 < HT; m0 += MB) {
                f32x4 w[2][MB];
#pragma unroll
                for (int mm = 0; mm < MB; ++mm) w[0][mm] = lds4(base + (m0 + mm) * 1024);
#pragma unroll
                for (int kq = 0; kq < HT; ++kq) {
                    const int cb = kq & 1;
                    if (kq + 1 < HT) {
#pragma unroll
                        for (int mm = 0; mm < MB; ++mm)
                            w[cb ^ 1][mm] = lds4(base + ((kq + 1) * HT + m0 + mm) * 1024);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int mm = 0; mm < MB; ++mm)
#pragma unroll
                            for (int tt = 0; tt < T; ++tt)
                                acc[tt][m0 + mm] = mfma4(w[cb][mm][r], h[tt][kq][r], acc[tt][m0 + mm]);
                }
            }
        } else if (HT >= 8 && D.mt <= 2) {
            // narrow output Dense of a wide net (<= 32 outputs): two tiles at most
            const int kb = C.kq_begin, ke = C.kq_end;
#pragma unroll
            for (int kq = 0; kq < HT; ++kq) {
                if (kq >= kb && kq < ke) {
                    const uint8_t* bq = base + (kq - kb) * D.mt * 1024;
                    const f32x4 w0 = lds4(bq);
                    if (D.mt == 2) {
                        const f32x4 w1 = lds4(bq + 1024);
#pragma unroll
                        for (int r = 0; r < 4; ++r)
#pragma unroll
                            for (int tt = 0; tt < T; ++tt) {
                                acc[tt][0] = mfma4(w0[r], h[tt][kq][r], acc[tt][0]);
                                acc[tt][1] = mfma4(w1[r], h[tt][kq][r], acc[tt][1]);
                            }
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
#pragma unroll
                            for (int tt = 0; tt < T; ++tt) acc[tt][0] = mfma4(w0[r], h[tt][kq][r], acc[tt][0]);
                    }
                }
            }
        } else if (D.mt == HT) {
            // full-M hidden Dense streamed in K-chunks (wide nets: one chunk per stage):
            // a uniform scalar guard per k-quad, no per-tile guards, MB interleaved
            // accumulators, fragments of the next m-group read ahead.
            constexpr int MB = HT < 4 ? HT : 4;
            const int kb = C.kq_begin, ke = C.kq_end;
#pragma unroll
            for (int kq = 0; kq < HT; ++kq) {
                if (kq >= kb && kq < ke) {
                    const uint8_t* bq = base + (kq - kb) * HT * 1024;
                    f32x4 w[2][MB];
#pragma unroll
                    for (int mm = 0; mm < MB; ++mm) w[0][mm] = lds4(bq + mm * 1024);
#pragma unroll
                    for (int m0 = 0; m0 < HT; m0 += MB) {
                        const int cb = (m0 / MB) & 1;
                        if (m0 + MB < HT) {
#pragma unroll
                            for (int mm = 0; mm < MB; ++mm) w[cb ^ 1][mm] = lds4(bq + (m0 + MB + mm) * 1024);
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r)
#pragma unroll
                            for (int mm = 0; mm < MB; ++mm)
#pragma unroll
                                for (int tt = 0; tt < T; ++tt)
                                    acc[tt][m0 + mm] = mfma4(w[cb][mm][r], h[tt][kq][r], acc[tt][m0 + mm]);
                    }
                }
            }
        } else {
#pragma unroll
            for (int kq = 0; kq < HT; ++kq) {
                if (kq >= C.kq_begin && kq < C.kq_end) {
                    const uint8_t* bq = base + (kq - C.kq_begin) * D.mt * 1024;
#pragma unroll
                    for (int m0 = 0; m0 < HT; m0 += MG) {
                        if (m0 < D.mt) {
                            f32x4 w[MG];
#pragma unroll
                            for (int mm = 0; mm < MG; ++mm)
                                w[mm] = (m0 + mm < D.mt) ? lds4(bq + (m0 + mm) * 1024) : f32x4{0, 0, 0, 0};
#pragma unroll
                            for (int r = 0; r < 4; ++r)
#pragma unroll
                                for (int mm = 0; mm < MG; ++mm)
                                    if (m0 + mm < HT && m0 + mm < D.mt)
#pragma unroll
                                        for (int tt = 0; tt < T; ++tt)
                                            acc[tt][m0 + mm] = mfma4(w[mm][r], h[tt][kq][r], acc[tt][m0 + mm]);
                        }
                    }
                }
            }
        }
    }

    // bias (after the product, as W*x .+ b) and activation
    ensure_stage(D.bias_stage, sg, a);
    if (D.has_bias) {
#pragma unroll
        for (int m = 0; m < HT; ++m) {
            if (m < D.mt) {
                const f32x4 b = lds4(sg.buf() + D.bias_lds + ((16 * m + 4 * g) << 2));
#pragma unroll
                for (int tt = 0; tt < T; ++tt) acc[tt][m] = acc[tt][m] + b;
            }
        }
    }
    if (D.act == DF_ACT_RELU) {
#pragma unroll
        for (int m = 0; m < HT; ++m)
#pragma unroll
            for (int tt = 0; tt < T; ++tt)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[tt][m][r] = relu(acc[tt][m][r]);
    } else if (D.act != DF_ACT_IDENTITY) {
#ifndef DF_NO_GENERIC_ACT
#pragma unroll
        for (int m = 0; m < HT; ++m) {
            if (m < D.mt) {
#pragma unroll
                for (int tt = 0; tt < T; ++tt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[tt][m][r] = act_fn(D.act, acc[tt][m][r]);
            }
        }
#endif
    }
}

// Evaluate one conditioner net (s or t) for this wave's T sample tiles into R.out.
template <int HT, int T, bool OUTV>
__device__ __forceinline__ void eval_net(const ChainArgs& a, const DevLayer& L, int dense0, int ndense,
                                         Stager& sg, const Smem& sm, const int (&rowoff)[T],
                                         NetRegs<HT, T, OUTV>& R, float* hs = nullptr, int64_t gs = -1) {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    const int32_t* feat = sm.tab + L.feat_tab;
    for (int k = 0; k < ndense; ++k) {
        const DevDense D = a.denses[dense0 + k];
        if (OUTV && k + 1 == ndense) {
            // ---- final Dense as a VALU GEMV: out[o] = Σ_k W[o][k] h[k] + b[o] ----
            ensure_stage(D.w3_stage, sg, a);
            const uint8_t* w3 = sg.buf() + D.w3_lds;
            const int inp = 16 * D.kt_in;
            const float* b3 = reinterpret_cast<const float*>(w3) + D.n_out * inp;
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                if (o < D.n_out) {
                    float p[T];
#pragma unroll
                    for (int tt = 0; tt < T; ++tt) p[tt] = 0.f;
#pragma unroll
                    for (int kq = 0; kq < HT; ++kq) {
                        if (kq < D.kt_in) {
                            f32x4 w = lds4(w3 + ((o * inp + 16 * kq + 4 * g) << 2));
#pragma unroll
                            for (int r = 0; r < 4; ++r)
#pragma unroll
                                for (int tt = 0; tt < T; ++tt) p[tt] = __builtin_fmaf(w[r], R.h[tt][kq][r], p[tt]);
                        }
                    }
#pragma unroll
                    for (int tt = 0; tt < T; ++tt) {
                        p[tt] += __shfl_xor(p[tt], 16);
                        p[tt] += __shfl_xor(p[tt], 32);
                        float v = p[tt];
                        if (D.has_bias) v = v + b3[o];
                        R.out[tt][0][o] = (D.act == DF_ACT_IDENTITY) ? v : act_fn(D.act, v);
                    }
                } else {
#pragma unroll
                    for (int tt = 0; tt < T; ++tt) R.out[tt][0][o] = 0.f;
                }
            }
            return;
        }
        dense_mfma<HT, T>(a, D, feat, sg, sm, rowoff, R.h, R.acc);
        if (k + 1 == ndense) {
            if constexpr (!OUTV) {
#pragma unroll
                for (int tt = 0; tt < T; ++tt)
#pragma unroll
                    for (int m = 0; m < out_tiles(HT); ++m) R.out[tt][m] = R.acc[tt][m];
            }
        } else {
#pragma unroll
            for (int tt = 0; tt < T; ++tt)
#pragma unroll
                for (int m = 0; m < HT; ++m) R.h[tt][m] = R.acc[tt][m];
            if (hs && gs >= 0) {  // training: keep H_k (post-activation), sample-major
                float* dst = hs + ((int64_t)k * a.batch + gs) * a.hsave_w + 4 * g;
#pragma unroll
                for (int m = 0; m < HT; ++m)
                    if (m < D.mt) *reinterpret_cast<f32x4*>(dst + 16 * m) = R.acc[0][m];
            }
        }
    }
}

__device__ __forceinline__ float sel4(const f32x4 v, int i) {
    float r = v[0];
    r = (i == 1) ? v[1] : r;
    r = (i == 2) ? v[2] : r;
    r = (i == 3) ? v[3] : r;
    return r;
}

enum Phase { PH_S_FWD, PH_T_FWD, PH_T_BWD, PH_S_BWD };

// Apply one coupling phase to the transformed dims of this wave's rows.
// Returns Σ_k s[k] for the s phases (0 otherwise).
template <int HT, int T, bool OUTV, int PH>
__device__ __forceinline__ void couple_phase(const NetRegs<HT, T, OUTV>& R, const DevLayer& L, const Smem& sm,
                                             const int (&rowoff)[T], float (&ssum)[T]) {
    const int g = (threadIdx.x & 63) >> 4;
    const int32_t* af = sm.tab + L.af_tab;
    constexpr bool SPH = (PH == PH_S_FWD || PH == PH_S_BWD);
    if constexpr (OUTV) {
        // every lane holds out[0..3]; lane group g transforms dim axis_af[g]
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
            const float y = sel4(R.out[tt][0], g);
            if (g < L.n_af) {
                const int slot = af[g];
                float v = sm.state[rowoff[tt] + slot];
                if (PH == PH_S_FWD) v = v * expf(y);
                if (PH == PH_T_FWD) v = v + y;
                if (PH == PH_T_BWD) v = v - y;
                if (PH == PH_S_BWD) v = v * expf(-y);
                sm.state[rowoff[tt] + slot] = v;
            }
            if (SPH) {
                // ldj = Σ_k s[k] in row order (RNVP.jl:180 / :86)
                float l = R.out[tt][0][0];
#pragma unroll
                for (int o = 1; o < 4; ++o)
                    if (o < L.n_af) l = l + R.out[tt][0][o];
                ssum[tt] = l;
            }
        }
    } else {
        constexpr int OT = out_tiles(HT);
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
            float p = 0.f;
#pragma unroll
            for (int m = 0; m < OT; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int o = 16 * m + 4 * g + r;
                    if (o < L.n_af) {
                        const int slot = af[o];
                        const float y = R.out[tt][m][r];
                        float v = sm.state[rowoff[tt] + slot];
                        if (PH == PH_S_FWD) v = v * expf(y);
                        if (PH == PH_T_FWD) v = v + y;
                        if (PH == PH_T_BWD) v = v - y;
                        if (PH == PH_S_BWD) v = v * expf(-y);
                        sm.state[rowoff[tt] + slot] = v;
                        if (SPH) p = p + y;
                    }
                }
            if (SPH) {
                p += __shfl_xor(p, 16);
                p += __shfl_xor(p, 32);
                ssum[tt] = p;
            }
        }
    }
}

}  // namespace impl

template <int HT, int MODE, bool OUTV>
__global__ void __launch_bounds__(kBlockThreads, DF_WAVES_PER_EU(HT))
chain_kernel(ChainArgs a) {
    using namespace impl;
    constexpr int T = 1;  // 16-sample MFMA column tiles held in registers at a time
    constexpr bool FWD = (MODE == MODE_FWD || MODE == MODE_FWD_INPLACE);
    constexpr bool WANT_LDJ = (MODE != MODE_FWD_INPLACE);

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Smem sm;
    const int stage_area = a.stage_bytes * a.n_stage_bufs;
    int32_t* tab = reinterpret_cast<int32_t*>(smem + stage_area);
    sm.tab = tab;
    sm.state = reinterpret_cast<float*>(smem + stage_area + a.tab_bytes);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int d = a.d, n = a.n, stride = a.stride, nd = n + d;
    const int nt = a.tiles;                 // 16-sample tiles per wave resident in LDS
    const int S = kWavesPerBlock * 16 * nt; // samples per workgroup
    const int cA = nd + 1, cE = nd + 2;     // state columns: chain ldj, element ldj
    const int64_t s0 = (int64_t)blockIdx.x * S;
    const int nvalid = (int)((a.batch - s0) < S ? (a.batch - s0) : S);

    Stager sg;
    sg.base = smem;
    sg.bytes = a.stage_bytes;
    sg.sched = FWD ? a.sched_fwd : a.sched_bwd;
    sg.n = FWD ? a.n_sched_fwd : a.n_sched_bwd;
    stager_start(sg, a);  // first stage's DMA overlaps the state load below

    // ---- tables, state tile [θ | z | 0 | ldj_chain | ldj_elem] ----
    for (int i = tid; i < a.tab_ints; i += kBlockThreads) tab[i] = a.tables[i];
    for (int i = tid; i < S * d; i += kBlockThreads) {
        const int smp = i / d, c = i - smp * d;
        float v = 0.f;
        if (smp < nvalid) v = a.zin[(s0 + smp) * d + c];
        sm.state[smp * stride + n + c] = v;
    }
    for (int i = tid; i < S * n; i += kBlockThreads) {
        const int smp = i / n, c = i - smp * n;
        float v = 0.f;
        if (smp < nvalid) {
            v = a.theta[(s0 + smp) * n + c];
            if (a.tmin) {  // normalize_input: (θ - θmin) ./ (θmax - θmin), 0 where max == min (Data.jl:213-218)
                const float lo = a.tmin[c], diff = a.tmax[c] - lo;
                v = (diff == 0.f) ? 0.f : (v - lo) / diff;
            }
        }
        sm.state[smp * stride + c] = v;
    }
    for (int i = tid; i < S; i += kBlockThreads)
        for (int c = nd; c < stride; ++c) sm.state[i * stride + c] = 0.f;
    __syncthreads();

    // row of lane (j, g) in tile tt of this wave
    auto row_of = [&](int tt) { return ((wave * nt + tt) * 16 + j) * stride; };

    // FlowElement grouping of ldj: CouplingBlock ldj_1 .+ ldj_2 (Blocks.jl:136,149),
    // chain left fold ldj .+ ldj_i (Chains.jl:160,179).  Lane group 0 owns the columns.
    bool have_acc = false;
    auto ldj_update = [&](int ro, float l, bool first_in_elem, bool last_in_elem) {
        if (!WANT_LDJ || g != 0) return;
        const float e = first_in_elem ? l : sm.state[ro + cE] + l;
        sm.state[ro + cE] = e;
        if (last_in_elem) sm.state[ro + cA] = have_acc ? sm.state[ro + cA] + e : e;
    };

    NetRegs<HT, T, OUTV> R;
    for (int it = 0; it < a.n_layers; ++it) {
        const int li = FWD ? it : a.n_layers - 1 - it;
        const DevLayer L = a.layers[li];
        const bool first_in_elem = FWD ? L.elem_start : L.elem_end;
        const bool last_in_elem = FWD ? L.elem_end : L.elem_start;
        if (L.kind == DF_LAYER_NORM) {
            // NormalizationLayer, src/norm/Normalization.jl:64-103
            const float al = L.alpha, be = L.beta, delta = be - al;
            const float* xmn = a.params + L.norm_off;
            const float* xmx = xmn + d;
            for (int tt = 0; tt < nt; ++tt) {
                const int ro = row_of(tt);
                for (int i = g; i < d; i += 4) {
                    const float lo = xmn[i], hi = xmx[i], xd = hi - lo;
                    float v = sm.state[ro + n + i];
                    if (FWD) v = ((xd * v - al * hi) + be * lo) / delta;
                    else v = (be * (v - lo) + al * (hi - v)) / xd;
                    sm.state[ro + n + i] = v;
                }
                ldj_update(ro, FWD ? L.ldj_const : -L.ldj_const, first_in_elem, last_in_elem);
            }
        } else {
            const bool rnvp = (L.kind == DF_LAYER_RNVP);
            float ssum[T];
            int rowoff[T];
            if (FWD) {
                if (rnvp) {
                    for (int tt = 0; tt < nt; ++tt) {
                        rowoff[0] = row_of(tt);
                        eval_net<HT, T, OUTV>(a, L, L.s_dense0, L.s_ndense, sg, sm, rowoff, R);
                        couple_phase<HT, T, OUTV, PH_S_FWD>(R, L, sm, rowoff, ssum);
                        ldj_update(rowoff[0], ssum[0], first_in_elem, last_in_elem);
                    }
                }
                for (int tt = 0; tt < nt; ++tt) {
                    rowoff[0] = row_of(tt);
                    eval_net<HT, T, OUTV>(a, L, L.t_dense0, L.t_ndense, sg, sm, rowoff, R);
                    couple_phase<HT, T, OUTV, PH_T_FWD>(R, L, sm, rowoff, ssum);
                    if (!rnvp) ldj_update(rowoff[0], 0.f, first_in_elem, last_in_elem);
                }
            } else {
                float* hs_t = nullptr;
                float* hs_s = nullptr;
                if (a.hsave) {
                    hs_s = a.hsave + (int64_t)(2 * li) * a.hsave_h * a.batch * a.hsave_w;
                    hs_t = hs_s + (int64_t)a.hsave_h * a.batch * a.hsave_w;
                }
                auto gs_of = [&](int tt) -> int64_t {
                    const int smp = (wave * nt + tt) * 16 + j;
                    return smp < nvalid ? s0 + smp : -1;
                };
                for (int tt = 0; tt < nt; ++tt) {
                    rowoff[0] = row_of(tt);
                    eval_net<HT, T, OUTV>(a, L, L.t_dense0, L.t_ndense, sg, sm, rowoff, R, hs_t, gs_of(tt));
                    couple_phase<HT, T, OUTV, PH_T_BWD>(R, L, sm, rowoff, ssum);
                    if (!rnvp) ldj_update(rowoff[0], 0.f, first_in_elem, last_in_elem);
                }
                if (rnvp) {
                    for (int tt = 0; tt < nt; ++tt) {
                        rowoff[0] = row_of(tt);
                        eval_net<HT, T, OUTV>(a, L, L.s_dense0, L.s_ndense, sg, sm, rowoff, R, hs_s, gs_of(tt));
                        couple_phase<HT, T, OUTV, PH_S_BWD>(R, L, sm, rowoff, ssum);
                        ldj_update(rowoff[0], -ssum[0], first_in_elem, last_in_elem);  // ln_det_jac = -Σ s
                    }
                }
            }
        }
        have_acc = have_acc || last_in_elem;
        if (!FWD && a.snap) {  // training: keep every layer's output for the reverse sweep
            float* dst = a.snap + (int64_t)li * a.batch * d;
            for (int tt = 0; tt < nt; ++tt) {
                const int smp = (wave * nt + tt) * 16 + j;
                if (smp < nvalid)
                    for (int i = g; i < d; i += 4) dst[(s0 + smp) * d + i] = sm.state[row_of(tt) + n + i];
            }
        }
    }

    // ---- epilogue ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no stage DMA may still target LDS
    if (MODE == MODE_LOGPDF) {
        // logpdf(MvNormal(0, I), z) .+ ldj = (c0 - Σ z²/2) + ldj   (Flows.jl:279)
        double part = 0.0;
        if (g == 0) {
            for (int tt = 0; tt < nt; ++tt) {
                const int ro = row_of(tt);
                const int smp = (wave * nt + tt) * 16 + j;
                float q = 0.f;
                for (int i = 0; i < d; ++i) {
                    const float zz = sm.state[ro + n + i];
                    q = q + zz * zz;
                }
                const float lp = (a.c0 - q / 2.f) + sm.state[ro + cA];
                if (smp < nvalid) {
                    if (a.lp_out) a.lp_out[s0 + smp] = lp;
                    part += (double)lp;
                }
            }
        }
        if (a.partial) {
            // deterministic workgroup reduction in fp64
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
        if (!a.xout) return;
    }
    __syncthreads();
    for (int i = tid; i < S * d; i += kBlockThreads) {
        const int smp = i / d, c = i - smp * d;
        if (smp < nvalid) a.xout[(s0 + smp) * d + c] = sm.state[smp * stride + n + c];
    }
    if (WANT_LDJ && MODE != MODE_LOGPDF && a.ldj_out) {
        for (int i = tid; i < nvalid; i += kBlockThreads) a.ldj_out[s0 + i] = sm.state[i * stride + cA];
    }
}

// ---------------------------------------------------------------------------
// per-variant host launchers
// ---------------------------------------------------------------------------
template <int HT>
void* chain_kernel_ptr(int mode, bool outv) {
#define DF_K(M) (outv ? reinterpret_cast<void*>(&chain_kernel<HT, M, true>) \
                      : reinterpret_cast<void*>(&chain_kernel<HT, M, false>))
    switch (mode) {
        case MODE_FWD: return DF_K(MODE_FWD);
        case MODE_FWD_INPLACE: return DF_K(MODE_FWD_INPLACE);
        case MODE_BWD: return DF_K(MODE_BWD);
        default: return DF_K(MODE_LOGPDF);
    }
#undef DF_K
}

template <int HT>
hipError_t launch_chain_ht(int mode, bool outv, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st) {
    void* f = chain_kernel_ptr<HT>(mode, outv);
    void* args[] = {const_cast<ChainArgs*>(&a)};
    return hipLaunchKernel(f, dim3(grid), dim3(kBlockThreads), args, lds, st);
}

template <int HT>
hipError_t chain_occupancy_ht(int mode, bool outv, size_t lds, int* blocks) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, chain_kernel_ptr<HT>(mode, outv), kBlockThreads, lds);
}

template <int HT>
hipError_t set_lds_limit_ht(size_t lds) {
    for (int mode = 0; mode < 4; ++mode)
        for (int ov = 0; ov < 2; ++ov) {
            hipError_t e = hipFuncSetAttribute(chain_kernel_ptr<HT>(mode, ov != 0),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

}  // namespace df
