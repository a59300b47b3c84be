// df_wide_impl.h — the wide-net chain kernel: every conditioner is the default
// _dflt_net shape at hidden width 256 (src/Layers.jl:33-50):
//   Dense(in <= 64, 256, relu) → Dense(256, 256, relu) → Dense(256, out <= 32)
// (the default σ; other activations run on the generic kernel).
// BASELINE configs 4/5 (d = 32, n = 8, hidden 256).
//
// Why a separate kernel: at hidden 256 one 16-sample tile needs 64 registers of
// activations plus 64 of accumulators, so the generic kernel (8 waves, 2 per SIMD,
// 256 registers each) holds ONE tile per wave and every 64 KiB weight stage feeds
// 128 samples per CU.  Here a workgroup is 4 waves — one per SIMD, 512 registers
// each (accumulators in AGPRs) — and each wave keeps 3 tiles resident, so a stage
// feeds 192 samples and every A-fragment read feeds 12 MFMAs instead of 4.  The
// weights live in their own blob of fixed 32 KiB stages (first Dense, 8 hidden
// stages, output Dense), double-buffered in LDS by global→LDS DMA in a fixed
// order, so every k-quad index is a compile-time constant (no guards, no
// dynamic register indexing).  Numerics as the other kernels: -ffp-contract=off,
// bias after the product, exact MFMA fma chains, same relu/exp.
#pragma once

#include "df_chain_impl.h"
#include "df_uniform_impl.h"

namespace df {
namespace wide {

using impl::lds4;
using impl::mfma4;

constexpr int kThreads = kWideWaves * 64;
constexpr int T = kWideT;

// Loads through the constant address space: scalar (s_load) instead of vector
// loads, so they never join the in-order vmcnt queue of the in-flight stage DMAs
// (the host writes these arrays before the launch; the kernel never stores to them).
template <class V>
__device__ __forceinline__ const V& cref(const V* p) {
    return *(const V*)(const __attribute__((address_space(4))) V*)(uintptr_t)p;
}

#ifndef DF_WIDE_SBIAS
#define DF_WIDE_SBIAS 0
#endif
// timing diagnostics of the SPLIT kernel (wrong results): bit 0 = no Dense epilogues
// (relu / hi + lo), bit 1 = no activation splits (chunk 0's planes reused), bit 2 = no
// stage waits / barriers
#ifndef DF_WIDE_DIAG
#define DF_WIDE_DIAG 0
#endif
// Bias rows 16m + 4g + r of lane group g: a vector load, or (DF_WIDE_SBIAS) 16
// scalar-loaded floats selected per lane group.
__device__ __forceinline__ f32x4 bias4(const float* b, int m) {
    const int g = (threadIdx.x & 63) >> 4;
    if (!DF_WIDE_SBIAS) return *reinterpret_cast<const f32x4*>(b + 16 * m + 4 * g);
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = cref(b + 16 * m + i);
    f32x4 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = g == 0 ? v[q] : g == 1 ? v[4 + q] : g == 2 ? v[8 + q] : v[12 + q];
    return r;
}

struct WStager {
    uint8_t* base;
    const int32_t* sched;
    int n;
    int idx;
    int cur;
    int bytes;  // ring slot size: kWideStageBytes, or kWideSplitStageBytes (SPLIT)
    int nb;     // ring slots: kWideBufs, or kWideSplitBufs (SPLIT)
    // staggered DMA (SPLIT): this wave's pieces of the next stage, issued one per
    // m-tile by split_chunk instead of all at the stage switch
    const uint8_t* blob;
    int psrc;   // byte offset of the pending stage in the blob
    int pdst;   // its ring slot's byte offset from base
    int pnext, pend;
    __device__ __forceinline__ uint8_t* buf() const { return slot(idx); }
    __device__ __forceinline__ uint8_t* slot(int i) const { return base + (i % nb) * bytes; }
    template <int NW>
    __device__ __forceinline__ void issue_one() {
        if (pnext < pend) {
            const int lane = threadIdx.x & 63;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(blob + psrc + (pnext << 10) + lane * 16),
                                             (__attribute__((address_space(3))) void*)(base + pdst + (pnext << 10)), 16,
                                             0, 0);
            pnext += NW;
        }
    }
    template <int NW>
    __device__ __forceinline__ void issue_all() {
        while (pnext < pend) issue_one<NW>();
    }
};

// DMA instructions wave w issues for a stage of `bytes` (1 KiB per instruction,
// chunks dealt round-robin over the waves).
template <int NW>
__device__ __forceinline__ int dma_ops(int bytes, int wave) {
    const int nchunk = bytes >> 10;
    return nchunk > wave ? (nchunk - wave + NW - 1) / NW : 0;
}

// s_waitcnt vmcnt(k) with k a run-time value (the count must be an immediate).
__device__ __forceinline__ void wait_vmcnt(int k) {
    switch (k) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
        case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
        case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    }
}

template <int NW>
__device__ __forceinline__ void dma(const ChainArgs& a, int s, uint8_t* dst) {
    const DevStage& st = cref(a.stages + s);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint8_t* src = a.blob + st.src_off;
    const int nchunk = st.bytes >> 10;
    for (int c = wave; c < nchunk; c += NW)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (c << 10) + lane * 16),
                                         (__attribute__((address_space(3))) void*)(dst + (c << 10)), 16, 0, 0);
}

// Stage s, which is the next one of the fixed schedule, becomes resident; the one
// kWideBufs − 1 places after it is put in flight into the ring slot just freed.
// Vector-memory loads return in order, so waiting until at most the newer
// in-flight stages' DMA instructions of this wave are outstanding means this
// wave's part of stage s has landed; the barrier then covers every wave's part.
template <int NW = kWideWaves, bool STAGGER = false, int NB = kWideBufs>
__device__ __forceinline__ void ensure(int s, WStager& sg, const ChainArgs& a) {
    if (s == sg.cur) return;
    if (STAGGER) sg.issue_all<NW>();  // pending pieces (of the newest stage in flight) not issued yet
    const int nidx = sg.idx + 1;
    if (NB > 2) {  // the NB − 2 newer stages' pieces may stay in flight (issued in order after stage s's)
        const int wave = threadIdx.x >> 6;
        int newer = 0;
        for (int q = 1; q < NB - 1; ++q)
            if (nidx + q < sg.n) newer += dma_ops<NW>(cref(a.stages + cref(sg.sched + nidx + q)).bytes, wave);
        wait_vmcnt(newer);
    } else if (!(DF_WIDE_DIAG & 4)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // A bare s_barrier: __syncthreads()'s release fence would also wait for the
    // newer stages' DMA (vmcnt(0)).  The stage ring is the only LDS data shared
    // between waves here, and each wave's reads of the slot being refilled have
    // returned (lgkmcnt(0)) before it arrives.
    if (!(DF_WIDE_DIAG & 4)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    sg.idx = nidx;
    sg.cur = s;
    if (nidx >= sg.n || cref(sg.sched + nidx) != s) {  // off schedule (never produced by the planner)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const DevStage st = a.stages[s];
        const f32x4* src = reinterpret_cast<const f32x4*>(a.blob + st.src_off);
        f32x4* dst = reinterpret_cast<f32x4*>(sg.buf());
        for (int i = threadIdx.x; i < (st.bytes >> 4); i += NW * 64) dst[i] = src[i];
        __syncthreads();
        sg.n = 0;
        return;
    }
    if (nidx + NB - 1 < sg.n) {
        if (STAGGER) {
            const DevStage& st = cref(a.stages + cref(sg.sched + nidx + NB - 1));
            sg.psrc = (int)st.src_off;
            sg.pdst = (int)(sg.slot(nidx + NB - 1) - sg.base);
            sg.pnext = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            sg.pend = st.bytes >> 10;
        } else {
            dma<NW>(a, cref(sg.sched + nidx + NB - 1), sg.slot(nidx + NB - 1));
        }
    }
}

// h = σ.(acc .+ b)  (b: 256 floats in global memory, L2-resident)
__device__ __forceinline__ void bias_act(const float* b, int act, const f32x4 (&acc)[T][16], f32x4 (&h)[T][16]) {
    const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const f32x4 bb = bias4(b, m);  // always present (zeros without a bias, df_plan.cpp)
#pragma unroll
        for (int t = 0; t < T; ++t) {
            f32x4 v = acc[t][m] + bb;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = uni::relu_fast(v[r]);  // planner: σ0 = σ1 = relu
            h[t][m] = v;
        }
    }
}

// Evaluate net N for this wave's T tiles (state rows ro[t]) into out[t][0..1]
// (rows 16m + 4g + r).  hs: training, keep H0 / H1 (sample-major, width hsave_w).
__device__ __forceinline__ void eval_net(const ChainArgs& a, const WNet& N, const int32_t* feat,
                                         const float* state, const int (&ro)[T], WStager& sg, f32x4 (&out)[T][2],
                                         float* hs, const int64_t (&gs)[T]) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    f32x4 h[T][16], acc[T][16];

    // ---- first Dense: features vcat(θ, z)[axis_nn] from the LDS state, k = 4s + g ----
    // (the first k-step, which always exists, starts every chain from an inline 0:
    // no accumulator zeroing)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
        if (st < N.nst0) {
            ensure(N.stage0 + st, sg, a);
            const uint8_t* buf = sg.buf() + lane * 16;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int kq = 2 * st + kk;
                const int rmax = N.ks - 4 * kq;  // k-steps of this k-quad carrying features
                if (rmax > 0) {
                    float xin[T][4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int slot = (r < rmax) ? feat[4 * (4 * kq + r) + g] : 0;
#pragma unroll
                        for (int t = 0; t < T; ++t) xin[t][r] = (r < rmax) ? state[ro[t] + slot] : 0.f;
                    }
#pragma unroll
                    for (int m0 = 0; m0 < 16; m0 += 4) {
                        f32x4 w[4];
#pragma unroll
                        for (int mm = 0; mm < 4; ++mm) w[mm] = lds4(buf + (kk * 16 + m0 + mm) * 1024);
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (r < rmax)
#pragma unroll
                                for (int mm = 0; mm < 4; ++mm)
#pragma unroll
                                    for (int t = 0; t < T; ++t)
                                        acc[t][m0 + mm] = mfma4(w[mm][r], xin[t][r],
                                                                (st == 0 && kk == 0 && r == 0)
                                                                    ? f32x4{0.f, 0.f, 0.f, 0.f}
                                                                    : acc[t][m0 + mm]);
                    }
                }
            }
        }
    }
    bias_act(a.wbias + N.b0, N.act0, acc, h);

    // ---- hidden Dense 256×256: 8 stages of 2 k-quads (chains start from an inline 0) ----
#pragma unroll
    for (int st = 0; st < 8; ++st) {
        ensure(N.stage0 + N.nst0 + st, sg, a);
        if (hs && st == 0) {  // training: keep H0.  Stored after the stage switch, so the
                              // stores drain under this stage's MFMAs, not at its vmcnt(0);
                              // streaming (non-temporal) so they do not evict the weights from L2
#pragma unroll
            for (int t = 0; t < T; ++t)
                if (gs[t] >= 0)
#pragma unroll
                    for (int m = 0; m < 16; ++m)
                        __builtin_nontemporal_store(h[t][m], reinterpret_cast<f32x4*>(hs + gs[t] * a.hsave_w + 16 * m + 4 * g));
        }
        const uint8_t* buf = sg.buf() + lane * 16;
        // 8 groups (k-quad kk, m-tiles m0..m0+3) per stage; group q+1's fragments are
        // read while group q's 32 MFMAs run (one wave per SIMD: nothing else would
        // hide the LDS latency)
        f32x4 wc[4], wn[4];
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) wc[mm] = lds4(buf + mm * 1024);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int kk = q >> 2, m0 = 4 * (q & 3), kq = 2 * st + kk;
            if (q + 1 < 8) {
                const int kk1 = (q + 1) >> 2, m1 = 4 * ((q + 1) & 3);
#pragma unroll
                for (int mm = 0; mm < 4; ++mm) wn[mm] = lds4(buf + (kk1 * 16 + m1 + mm) * 1024);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int mm = 0; mm < 4; ++mm)
#pragma unroll
                    for (int t = 0; t < T; ++t)
                        acc[t][m0 + mm] = mfma4(wc[mm][r], h[t][kq][r],
                                                (st == 0 && kk == 0 && r == 0) ? f32x4{0.f, 0.f, 0.f, 0.f}
                                                                               : acc[t][m0 + mm]);
#pragma unroll
            for (int mm = 0; mm < 4; ++mm) wc[mm] = wn[mm];
        }
    }
    bias_act(a.wbias + N.b1, N.act1, acc, h);

    // ---- output Dense (<= 32 outputs): [kq < 16][m < mto] ----
    ensure(N.stage0 + N.nst0 + 8, sg, a);
    if (hs) {  // training: keep H1 (after the stage switch, as H0)
        float* hs1 = hs + a.batch * a.hsave_w;
#pragma unroll
        for (int t = 0; t < T; ++t)
            if (gs[t] >= 0)
#pragma unroll
                for (int m = 0; m < 16; ++m)
                    __builtin_nontemporal_store(h[t][m], reinterpret_cast<f32x4*>(hs1 + gs[t] * a.hsave_w + 16 * m + 4 * g));
    }
    const uint8_t* buf = sg.buf() + lane * 16;
#pragma unroll
    for (int t = 0; t < T; ++t) out[t][0] = out[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (N.mto == 2) {
#pragma unroll
        for (int kq = 0; kq < 16; ++kq) {
            const f32x4 w0 = lds4(buf + (kq * 2) * 1024), w1 = lds4(buf + (kq * 2 + 1) * 1024);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    out[t][0] = mfma4(w0[r], h[t][kq][r], out[t][0]);
                    out[t][1] = mfma4(w1[r], h[t][kq][r], out[t][1]);
                }
        }
    } else {
        f32x4 w0 = lds4(buf);
#pragma unroll
        for (int kq = 0; kq < 16; ++kq) {
            const f32x4 wq = w0;
            if (kq + 1 < 16) w0 = lds4(buf + (kq + 1) * 1024);  // next k-quad in flight
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int t = 0; t < T; ++t) out[t][0] = mfma4(wq[r], h[t][kq][r], out[t][0]);
        }
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        if (m < N.mto) {
            const f32x4 bb = bias4(a.wbias + N.bo, m);
#pragma unroll
            for (int t = 0; t < T; ++t) out[t][m] = out[t][m] + bb;  // planner: σo = identity
        }
    }
}

// ---- SPLIT variant: every Dense as bf16x3 products on bf16 MFMA (df_uniform_impl.h) ----
using uni::bf16x8;
using uni::mfma_bf;
using uni::split8;
#ifndef DF_WSPLIT_WAVES
#define DF_WSPLIT_WAVES 4
#endif
constexpr int kSplitWaves = DF_WSPLIT_WAVES;         // 4: one wave per SIMD, 2 tiles; 8: two, 1 tile
constexpr int kSplitT = 8 / DF_WSPLIT_WAVES;        // 128 samples per workgroup either way
#ifndef DF_WIDE_STAGGER
#define DF_WIDE_STAGGER 1
#endif
#ifndef DF_WIDE_PF
#define DF_WIDE_PF 1
#endif

// acc += W·x over one 32-input chunk for m-tiles [0, MT): planes [m][p][lane][8] at
// buf (lane offset applied), activation planes x[t][p]; the next m-tile's planes
// are read while this one's 6·TT MFMAs run.
//   HILO: the leading product w0·x0 goes to hi, the five correction products
//   (small terms first) to lo.  Inside one MFMA a sum of products is truncated
//   toward zero (tools/probe/mfma_round.hip: C + ONE product rounds to nearest
//   even, several do not), so a running total fed back as the C operand six times
//   per chunk took a biased rounding each time: at config 4 (eight chunks) that
//   doubled the 99th-percentile error against the exact-f32 kernel.  With hi/lo
//   the total takes one per chunk and lo's are relative to the small terms.  hi
//   and lo are touched only by MFMAs (AGPR-resident); the caller adds them once.
//   !HILO (the one- or two-chunk first Dense): all six products onto hi.
template <int TT, int MT, bool HILO, int MA, int M0 = 0>
__device__ __forceinline__ void split_chunk(const uint8_t* buf, const bf16x8 (&x)[TT][3], f32x4 (&hi)[TT][MA],
                                            f32x4 (&lo)[TT][MA], WStager& sg) {
    // fragment ring, DF_WIDE_PF m-tiles ahead
    constexpr int PF = DF_WIDE_PF;
    bf16x8 w[PF + 1][3];
#pragma unroll
    for (int q = 0; q < PF; ++q)
        if (q < MT)
#pragma unroll
            for (int p = 0; p < 3; ++p) w[q][p] = *reinterpret_cast<const bf16x8*>(buf + q * 3072 + p * 1024);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int cb = m % (PF + 1);
        if (m + PF < MT) {
#pragma unroll
            for (int p = 0; p < 3; ++p)
                w[(m + PF) % (PF + 1)][p] = *reinterpret_cast<const bf16x8*>(buf + (m + PF) * 3072 + p * 1024);
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            f32x4 v = HILO ? lo[t][M0 + m] : hi[t][M0 + m];
            v = mfma_bf(w[cb][2], x[t][0], v);
            v = mfma_bf(w[cb][1], x[t][1], v);
            v = mfma_bf(w[cb][0], x[t][2], v);
            v = mfma_bf(w[cb][1], x[t][0], v);
            v = mfma_bf(w[cb][0], x[t][1], v);
            if (HILO) {
                lo[t][M0 + m] = v;
                hi[t][M0 + m] = mfma_bf(w[cb][0], x[t][0], hi[t][M0 + m]);
            } else {
                hi[t][M0 + m] = mfma_bf(w[cb][0], x[t][0], v);
            }
        }
        if (DF_WIDE_STAGGER) sg.issue_one<kSplitWaves>();  // one DMA piece of the next stage per m-tile
        asm volatile("" ::: "memory");  // fragment reads stay one m-tile ahead (no hoisting)
    }
}

// hi + lo of a hi/lo accumulator pair.  DF_WIDE_SADD: four v_add_f32 (asm) instead of the
// two v_pk_add_f32 plain -O3 makes of an f32x4 add (a packed f32 op issues at a quarter of
// the rate of v_add_f32 beside MFMAs, tools/probe/mfma_valu.hip); the same roundings.  On
// for the forward unit only (Makefile): config-4 forward 15.83 -> 15.73 M cycles, the
// logpdf / training-inverse unit lost 0.6% of the config-5 step (gpurun_out/r06n)
#ifndef DF_WIDE_SADD
#define DF_WIDE_SADD 0
#endif
__device__ __forceinline__ f32x4 add_hilo(const f32x4& a, const f32x4& b) {
    if constexpr (DF_WIDE_SADD) {
        f32x4 r;
#pragma unroll
        for (int q = 0; q < 4; ++q) asm("v_add_f32 %0, %1, %2" : "=v"(r[q]) : "v"(a[q]), "v"(b[q]));
        return r;
    }
    return a + b;
}

// Planes of accumulator tiles 2c, 2c+1 (inputs 32c + 16(e>>2) + 4g + (e&3)).
// DF_WIDE_MREM: the remainders on the matrix pipe (uni::split8_mrem, bitwise split8).  Off:
// this kernel is matrix-pipe bound at one wave per SIMD, and the extra 16x16x16 MFMAs cost
// more than the v_dot2c they replace (config-4 forward 35.7 vs 37.3 Msamples/s).
#ifndef DF_WIDE_MREM
#define DF_WIDE_MREM 0
#endif
template <int TT>
__device__ __forceinline__ void split_tiles(const f32x4 (&h)[TT][16], int c, bf16x8 (&x)[TT][3]) {
    const uni::short4v eye = uni::neg_eye();
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        if constexpr (DF_WIDE_MREM) {
            uni::split8_mrem(eye, h[t][2 * c], h[t][2 * c + 1], x[t][0], x[t][1], x[t][2]);
        } else {
            const float v[8] = {h[t][2 * c][0],     h[t][2 * c][1],     h[t][2 * c][2],     h[t][2 * c][3],
                                h[t][2 * c + 1][0], h[t][2 * c + 1][1], h[t][2 * c + 1][2], h[t][2 * c + 1][3]};
            split8(v, x[t][0], x[t][1], x[t][2]);
        }
    }
}

// eval_net on the SPLIT stages (layout: build_wide_split): accumulators start from
// the bias (b + W·x), relu after.
//   first Dense  ceil(in/32) stages [m < 16][p][lane][8], lane group g carries
//                features 32c + 8g + e
//   hidden Dense 8 stages [m < 16][p][lane][8], one 32-input chunk each (hi/lo)
//   output Dense one stage [c < 8][m < mto][p][lane][8] (hi/lo)
#ifndef DF_WSNAP_SPREAD
#define DF_WSNAP_SPREAD 1
#endif

// Training snapshot of a hidden activation (H0 or H1, rows of sample gs[t]) during
// 32-input chunk c of the Dense that consumes it. SPREAD: the chunk's own two m-tiles
// (its stores drain during the chunk's MFMAs; a stage switch waits vmcnt(0), so a
// 16-tile burst would stall the next one), else all 16 tiles at chunk 0.
template <int TT, bool SPREAD>
__device__ __forceinline__ void snapshot(const f32x4 (&h)[TT][16], float* dst, const int64_t (&gs)[TT], int w, int c) {
    const int g = (threadIdx.x & 63) >> 4;
    if (!SPREAD && c != 0) return;
#pragma unroll
    for (int t = 0; t < TT; ++t)
        if (gs[t] >= 0)
#pragma unroll
            for (int m = 0; m < 16; ++m)
                if (!SPREAD || (m >> 1) == c)
                    __builtin_nontemporal_store(h[t][m], reinterpret_cast<f32x4*>(dst + gs[t] * w + 16 * m + 4 * g));
}

template <int TT>
__device__ __forceinline__ void eval_net_split(const ChainArgs& a, const WNet& N, const int32_t* sfeat,
                                               const float* state, const int (&ro)[TT], WStager& sg,
                                               f32x4 (&out)[TT][2], float* hs, float* hs1, float* fs,
                                               const int64_t (&gs)[TT]) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    f32x4 h[TT][16], acc[TT][16], lo[TT][16];

    // ---- first Dense ----
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const f32x4 b = bias4(a.wbias + N.b0, m);
#pragma unroll
        for (int t = 0; t < TT; ++t) acc[t][m] = b;
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (kWideSplitHalves * c < N.nst0) {
            bf16x8 x[TT][3];
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = state[ro[t] + sfeat[32 * c + 8 * g + e]];
                split8(v, x[t][0], x[t][1], x[t][2]);
                if (fs && c == 0 && gs[t] >= 0) {  // training: the features (H0 is recomputed from them)
                    float* fp = fs + gs[t] * 32 + 8 * g;
                    __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(fp));
                    __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(fp + 4));
                }
            }
            ensure<kSplitWaves, DF_WIDE_STAGGER != 0, kWideSplitBufs>(N.stage0 + kWideSplitHalves * c, sg, a);
            split_chunk<TT, 16 / kWideSplitHalves, false, 16, 0>(sg.buf() + lane * 16, x, acc, acc, sg);
            if constexpr (kWideSplitHalves == 2) {
                ensure<kSplitWaves, DF_WIDE_STAGGER != 0, kWideSplitBufs>(N.stage0 + 2 * c + 1, sg, a);
                split_chunk<TT, 8, false, 16, 8>(sg.buf() + lane * 16, x, acc, acc, sg);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int m = 0; m < 16; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) h[t][m][r] = (DF_WIDE_DIAG & 1) ? acc[t][0][r] : uni::relu_fast(acc[t][m][r]);

    // ---- hidden Dense 256×256 ----
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const f32x4 b = bias4(a.wbias + N.b1, m);
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            acc[t][m] = b;
            lo[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        ensure<kSplitWaves, DF_WIDE_STAGGER != 0, kWideSplitBufs>(N.stage0 + N.nst0 + kWideSplitHalves * c, sg, a);
        bf16x8 x[TT][3];
        split_tiles<TT>(h, (DF_WIDE_DIAG & 2) ? 0 : c, x);
        if (hs) snapshot<TT, DF_WSNAP_SPREAD != 0>(h, hs, gs, a.hsave_w, c);  // training: keep H0 (as in eval_net)
        split_chunk<TT, 16 / kWideSplitHalves, true, 16, 0>(sg.buf() + lane * 16, x, acc, lo, sg);
        if constexpr (kWideSplitHalves == 2) {
            ensure<kSplitWaves, DF_WIDE_STAGGER != 0, kWideSplitBufs>(N.stage0 + N.nst0 + 2 * c + 1, sg, a);
            split_chunk<TT, 8, true, 16, 8>(sg.buf() + lane * 16, x, acc, lo, sg);
        }
    }
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const f32x4 v = (DF_WIDE_DIAG & 1) ? acc[t][m & 1] : add_hilo(acc[t][m], lo[t][m]);
#pragma unroll
            for (int r = 0; r < 4; ++r) h[t][m][r] = (DF_WIDE_DIAG & 1) ? v[r] : uni::relu_fast(v[r]);
        }

    // ---- output Dense (<= 32 outputs) ----
    ensure<kSplitWaves, DF_WIDE_STAGGER != 0, kWideSplitBufs>(N.stage0 + N.nst0 + 8 * kWideSplitHalves, sg, a);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const f32x4 b = m < N.mto ? bias4(a.wbias + N.bo, m) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            acc[t][m] = b;
            lo[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    const int so0 = N.stage0 + N.nst0 + 8 * kWideSplitHalves;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (N.nso == 2 && c == 4) ensure<kSplitWaves, DF_WIDE_STAGGER != 0, kWideSplitBufs>(so0 + 1, sg, a);
        const uint8_t* buf = sg.buf() + lane * 16;
        bf16x8 x[TT][3];
        split_tiles<TT>(h, (DF_WIDE_DIAG & 2) ? 0 : c, x);
        if (hs1) snapshot<TT, DF_WSNAP_SPREAD != 0>(h, hs1, gs, a.hsave_w, c);
        if (N.mto == 2) split_chunk<TT, 2, true>(buf + (c & (8 / N.nso - 1)) * 2 * 3072, x, acc, lo, sg);
        else split_chunk<TT, 1, true>(buf + c * 3072, x, acc, lo, sg);
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        out[t][0] = add_hilo(acc[t][0], lo[t][0]);
        out[t][1] = add_hilo(acc[t][1], lo[t][1]);
    }
}

// Coupling phase on the transformed dims (row o = 16m + 4g + r of out ↔ axis_af[o]);
// sum[t] = Σ_o s_o for the s phases.
template <int PH, int TT = T>
__device__ __forceinline__ void couple(const f32x4 (&out)[TT][2], const WLayer& L, const int32_t* tab, float* state,
                                       const int (&ro)[TT], float (&sum)[TT]) {
    const int g = (threadIdx.x & 63) >> 4;
    constexpr bool SPH = (PH == impl::PH_S_FWD || PH == impl::PH_S_BWD);
    const int32_t* af = tab + L.af_tab;
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        float p = 0.f;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = 16 * m + 4 * g + r;
                if (o < L.n_af) {
                    const int slot = af[o];
                    const float y = out[t][m][r];
                    state[ro[t] + slot] = uni::couple1<PH>(state[ro[t] + slot], y);
                    if (SPH) p = p + y;
                }
            }
        sum[t] = SPH ? uni::xgroup_sum(p) : 0.f;
    }
}

}  // namespace wide

template <int MODE, bool SPLIT = false>
__global__ void __launch_bounds__(SPLIT ? wide::kSplitWaves * 64 : wide::kThreads, 1) wide_kernel(ChainArgs a) {
    using namespace wide;
    constexpr bool FWD = (MODE == MODE_FWD || MODE == MODE_FWD_INPLACE);
    constexpr bool WANT_LDJ = (MODE != MODE_FWD_INPLACE);
    constexpr int SBYTES = SPLIT ? kWideSplitStageBytes : kWideStageBytes;
    constexpr int NW = SPLIT ? kSplitWaves : kWideWaves;  // waves
    constexpr int TT = SPLIT ? kSplitT : T;               // 16-sample tiles per wave
    constexpr int NT = NW * 64;

    ClockStamp clk;
    clk.begin(a);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NB = SPLIT ? kWideSplitBufs : kWideBufs;  // ring slots
    const int stage_area = NB * SBYTES;
    int32_t* tab = reinterpret_cast<int32_t*>(smem + stage_area);
    float* state = reinterpret_cast<float*>(smem + stage_area + a.tab_bytes);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int d = a.d, n = a.n, stride = a.stride, nd = n + d;
    constexpr int S = NW * 16 * TT;
    const int cA = nd + 1, cE = nd + 2;
    const int64_t s0 = (int64_t)blockIdx.x * S;
    const int nvalid = (int)((a.batch - s0) < S ? (a.batch - s0) : S);

    WStager sg;
    sg.base = smem;
    sg.sched = FWD ? a.sched_fwd : a.sched_bwd;
    sg.n = FWD ? a.n_sched_fwd : a.n_sched_bwd;
    sg.idx = -1;
    sg.cur = -1;
    sg.bytes = SBYTES;
    sg.nb = NB;
    sg.blob = a.blob;
    sg.psrc = sg.pdst = sg.pnext = sg.pend = 0;
    for (int q = 0; q < NB - 1 && q < sg.n; ++q) dma<NW>(a, cref(sg.sched + q), sg.slot(q));

    for (int i = tid; i < a.tab_ints; i += NT) tab[i] = a.tables[i];
    for (int i = tid; i < S * d; i += NT) {
        const int smp = i / d, c = i - smp * d;
        state[smp * stride + n + c] = (smp < nvalid) ? a.zin[(s0 + smp) * d + c] : 0.f;
    }
    for (int i = tid; i < S * n; i += NT) {
        const int smp = i / n, c = i - smp * n;
        float v = 0.f;
        if (smp < nvalid) {
            v = a.theta[(s0 + smp) * n + c];
            if (a.tmin) {  // normalize_input (Data.jl:213-218)
                const float lo = a.tmin[c], diff = a.tmax[c] - lo;
                v = (diff == 0.f) ? 0.f : (v - lo) / diff;
            }
        }
        state[smp * stride + c] = v;
    }
    for (int i = tid; i < S; i += NT)
        for (int c = nd; c < stride; ++c) state[i * stride + c] = 0.f;
    __syncthreads();

    int ro[TT];
    int64_t gs[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        const int smp = (wave * TT + t) * 16 + j;
        ro[t] = smp * stride;
        gs[t] = smp < nvalid ? s0 + smp : -1;
    }
    bool have_acc = false;
    auto ldj_update = [&](int r, float l, bool first_in_elem, bool last_in_elem) {
        if (!WANT_LDJ || g != 0) return;
        const float e = first_in_elem ? l : state[r + cE] + l;
        state[r + cE] = e;
        if (last_in_elem) state[r + cA] = have_acc ? state[r + cA] + e : e;
    };

    for (int it = 0; it < a.n_layers; ++it) {
        const int li = FWD ? it : a.n_layers - 1 - it;
        const WLayer& L = cref(a.wlayers + li);
        const bool first_in_elem = FWD ? L.elem_start : L.elem_end;
        const bool last_in_elem = FWD ? L.elem_end : L.elem_start;
        if (L.kind == DF_LAYER_NORM) {
            // NormalizationLayer, src/norm/Normalization.jl:64-103
            const float al = L.alpha, be = L.beta, delta = be - al;
            const float* xmn = a.params + L.norm_off;
            const float* xmx = xmn + d;
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                for (int i = g; i < d; i += 4) {
                    const float lo = xmn[i], hi = xmx[i], xd = hi - lo;
                    float v = state[ro[t] + n + i];
                    if (FWD) v = ((xd * v - al * hi) + be * lo) / delta;
                    else v = (be * (v - lo) + al * (hi - v)) / xd;
                    state[ro[t] + n + i] = v;
                }
                ldj_update(ro[t], FWD ? L.ldj_const : -L.ldj_const, first_in_elem, last_in_elem);
            }
        } else {
            const bool rnvp = (L.kind == DF_LAYER_RNVP);
            const int32_t* feat = tab + L.feat_tab;
            float* hs_s = nullptr;
            float* hs_t = nullptr;
            if (!FWD && a.hsave) {
                hs_s = a.hsave + (int64_t)(2 * li) * a.hsave_h * a.batch * a.hsave_w;
                hs_t = hs_s + (int64_t)a.hsave_h * a.batch * a.hsave_w;
            }
            auto run = [&](const WNet& N, auto ph_tag, float* hs, bool sphase, float sign) {
                constexpr int PH = decltype(ph_tag)::value;
                f32x4 out[TT][2];
                float sum[TT];
                if constexpr (SPLIT) {
                    // training snapshots: H0 and H1 at hs (hsave_h = 2), or with fsave the
                    // features and H1 only (hs is then the net's H1 slot, hsave_h = 1)
                    float* fs = nullptr;
                    if (hs && a.fsave) {
                        const int64_t slot = (hs - a.hsave) / (a.batch * a.hsave_w);
                        fs = a.fsave + slot * a.batch * 32;
                    }
                    float* h0 = (hs && !a.fsave) ? hs : nullptr;
                    float* h1 = hs ? (a.fsave ? hs : hs + a.batch * a.hsave_w) : nullptr;
                    eval_net_split<TT>(a, N, tab + L.pad0, state, ro, sg, out, h0, h1, fs, gs);
                } else {
                    eval_net(a, N, feat, state, ro, sg, out, hs, gs);
                }
                couple<PH, TT>(out, L, tab, state, ro, sum);
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    if (sphase) ldj_update(ro[t], sign * sum[t], first_in_elem, last_in_elem);
                    else if (!rnvp) ldj_update(ro[t], 0.f, first_in_elem, last_in_elem);
                }
            };
            using PSF = std::integral_constant<int, impl::PH_S_FWD>;
            using PTF = std::integral_constant<int, impl::PH_T_FWD>;
            using PTB = std::integral_constant<int, impl::PH_T_BWD>;
            using PSB = std::integral_constant<int, impl::PH_S_BWD>;
            if (FWD) {
                if (rnvp) run(L.s, PSF{}, nullptr, true, 1.f);
                run(L.t, PTF{}, nullptr, false, 1.f);
            } else {
                run(L.t, PTB{}, hs_t, false, 1.f);
                if (rnvp) run(L.s, PSB{}, hs_s, true, -1.f);  // ln_det_jac = -Σ s
            }
        }
        have_acc = have_acc || last_in_elem;
        if (!FWD && a.snap) {  // training: keep every layer's output for the reverse sweep
            float* dst = a.snap + (int64_t)li * a.batch * d;
#pragma unroll
            for (int t = 0; t < TT; ++t)
                if (gs[t] >= 0)
                    for (int i = g; i < d; i += 4) dst[gs[t] * d + i] = state[ro[t] + n + i];
        }
    }

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (MODE == MODE_LOGPDF) {
        double part = 0.0;
        if (g == 0) {
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                float q = 0.f;
                for (int i = 0; i < d; ++i) {
                    const float zz = state[ro[t] + n + i];
                    q = q + zz * zz;
                }
                const float lp = (a.c0 - q / 2.f) + state[ro[t] + cA];
                if (gs[t] >= 0) {
                    if (a.lp_out) a.lp_out[gs[t]] = lp;
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
                for (int w = 0; w < NW; ++w) s += red[w];
                a.partial[blockIdx.x] = s;
            }
        }
        if (!a.xout) {
            clk.end(a);
            return;
        }
    }
    __syncthreads();
    for (int i = tid; i < S * d; i += NT) {
        const int smp = i / d, c = i - smp * d;
        if (smp < nvalid) a.xout[(s0 + smp) * d + c] = state[smp * stride + n + c];
    }
    if (WANT_LDJ && MODE != MODE_LOGPDF && a.ldj_out) {
        for (int i = tid; i < nvalid; i += NT) a.ldj_out[s0 + i] = state[i * stride + cA];
    }
    clk.end(a);
}

}  // namespace df
