// df_ltrain.hip — kernels of the layer-wise training path (df_ltrain.h).
#include <utility>

#include "df_chain_impl.h"
#include "df_ltrain.h"
#include "df_train_impl.h"

namespace df {

namespace {

using impl::lds4;
using impl::mfma4;

// 8 values (two f32x4 of a lane, a then b) → their bf16x3 planes on the VALU (uni::split8:
// v_mov + v_dot2c per remainder).  DF_LT_MREM=1: the remainders on the matrix pipe
// (uni::split8_mrem, one v_mfma_f32_16x16x16_bf16 with A = −I per 4 values: an exact
// element-wise x − hi for any 4 values of a lane), bitwise the same planes; measured slower
// here (config-5 step 34.2 vs 33.4 ms, gpurun_out/r05m)
#ifndef DF_LT_MREM
#define DF_LT_MREM 0
#endif
#ifndef DF_LDENSE_MASK_PF
#define DF_LDENSE_MASK_PF 1
#endif
#ifndef DF_LDENSE_ZV_EARLY
#define DF_LDENSE_ZV_EARLY 1
#endif
#ifndef DF_LDW_MREM  // the split dW kernel's own choice (its matrix pipe idles in the split phase)
#define DF_LDW_MREM DF_LT_MREM
#endif
template <bool MREM = (DF_LT_MREM != 0)>
__device__ __forceinline__ void split8x(const f32x4& a, const f32x4& b, uni::bf16x8& p0, uni::bf16x8& p1,
                                        uni::bf16x8& p2) {
    if constexpr (MREM) {
        uni::split8_mrem(uni::neg_eye(), a, b, p0, p1, p2);
    } else {
        const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        uni::split8(v, p0, p1, p2);
    }
}

__device__ __forceinline__ float gather_feature(const LDenseArgs& a, int slot, int64_t s) {
    if (slot < a.n) {
        float v = a.theta[s * a.n + slot];
        if (a.tmin) {  // normalize_input (Data.jl:213-218)
            const float lo = a.tmin[slot], diff = a.tmax[slot] - lo;
            v = (diff == 0.f) ? 0.f : (v - lo) / diff;
        }
        return v;
    }
    if (slot < a.n + a.d) return a.u_in[s * a.d + (slot - a.n)];
    return 0.f;
}

// One Dense over the whole batch: acc = A · in, A = packed W or Wᵀ (16·MT rows),
// then the fused epilogue.  Persistent workgroups; each wave owns kLTiles
// 16-sample tiles per round; A is streamed through two LDS chunk buffers.
// SPLIT (LIN_BUF, MT = 16): A = a.sfrag, bf16x3 planes [c][m][p][lane][8] of 32-input
// chunks (lane (g, i): A[16m + i, 32c + 16(e>>2) + 4g + (e&3)]), the B rows split on
// the fly (df_uniform_impl.h), six products per chunk on bf16 MFMA onto the f32
// accumulators (gradients: the 1e-4 criterion of the training tests).
// NW waves of TT tiles each: the f32 instances 8 × kLTiles (two waves per SIMD); the SPLIT
// ones kSplitWaves × kSplitTiles — one wave per SIMD whose 4 × 16 accumulator tiles sit
// in the AGPR half of the register file, so every bf16x3 weight fragment read from LDS
// feeds 4 tiles' products instead of 2 (same samples per workgroup round).
template <int MT, int IN, int EPI, bool SPLIT = false, int NW = kWavesPerBlock, int TT = kLTiles>
__global__ void __launch_bounds__(NW * 64, 1) ldense_kernel(LDenseArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int T = TT;
    // LEPI_DACT_XBAR_MASK: LEPI_DACT_XBAR with σ'(H0) from the split dW1's relu mask
    // (a.hmask) — no σ' argument rows are loaded, so none are held in registers
    constexpr bool XB = (EPI == LEPI_DACT_XBAR || EPI == LEPI_DACT_XBAR_MASK);
    constexpr bool MASK = (EPI == LEPI_DACT_XBAR_MASK);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int chunk_bytes = SPLIT ? MT * 3072 : a.chunk_kq * MT * 1024;
    const int nchunks = SPLIT ? a.nkq / 2 : (a.nkq + a.chunk_kq - 1) / a.chunk_kq;
    const int64_t ntiles = (a.batch + 15) / 16;
    const int64_t per_round = (int64_t)gridDim.x * NW * T;
    const int64_t rounds = (ntiles + per_round - 1) / per_round;
    const int64_t total = rounds * nchunks;

    auto dma = [&](int c, uint8_t* dst) {
        if constexpr (SPLIT) {
            const uint8_t* src = a.sfrag + (size_t)c * MT * 3072;
            for (int q = wave; q < 3 * MT; q += NW)
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (q << 10) + lane * 16),
                                                 (__attribute__((address_space(3))) void*)(dst + (q << 10)), 16, 0,
                                                 0);
            return;
        }
        const int kq0 = c * a.chunk_kq;
        const int kq1 = (kq0 + a.chunk_kq < a.nkq) ? kq0 + a.chunk_kq : a.nkq;
        const uint8_t* src = a.wfrag + (size_t)kq0 * MT * 1024;
        const int nk = (kq1 - kq0) * MT;  // KiB
        for (int q = wave; q < nk; q += NW)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (q << 10) + lane * 16),
                                             (__attribute__((address_space(3))) void*)(dst + (q << 10)), 16, 0,
                                             0);
    };
    // after the chunk buffer(s): two full chunks, or the single (possibly short) one
    uint8_t* w0t_lds = smem + (nchunks > 1 ? 2 * chunk_bytes : SPLIT ? chunk_bytes : a.nkq * MT * 1024);
    if constexpr (XB) {  // W0ᵀ fragments stay resident for the x̄ product
        // f32 fragments, or (SPLIT, a.w0s) bf16x3 planes [c][m][p][lane][8] of 32-row chunks
        const int n16 = (SPLIT && a.w0s) ? (a.w0t_nkq / 2) * a.w0t_mt * 3 * 64 : a.w0t_mt * a.w0t_nkq * 64;
        const f32x4* src = reinterpret_cast<const f32x4*>((SPLIT && a.w0s) ? a.w0s : a.w0t);
        for (int q = threadIdx.x; q < n16; q += NW * 64) reinterpret_cast<f32x4*>(w0t_lds)[q] = src[q];
        // z̄ column of conditioner feature f (0xff: not an identity dim of z; d <= 64),
        // 64 bytes after the W0ᵀ fragments, fixed for the launch
        if (threadIdx.x < 64) {
            const int f = threadIdx.x;
            const int slot = f < a.n_in ? a.feat[f] : -1;
            w0t_lds[n16 * 16 + f] = (slot >= a.n && slot < a.n + a.d) ? (uint8_t)(slot - a.n) : (uint8_t)0xff;
        }
    }
    dma(0, smem);
    if (nchunks == 1 || XB) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    int64_t i = 0;
    for (int64_t r = 0; r < rounds; ++r) {
        const int64_t t0 = ((r * gridDim.x + blockIdx.x) * NW + wave) * T;
        int64_t smp[T];
        bool valid[T];
#pragma unroll
        for (int t = 0; t < T; ++t) {
            smp[t] = (t0 + t) * 16 + j;
            valid[t] = smp[t] < a.batch;
        }
        f32x4 acc[T][MT];
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};

        // B operand of k-quad kq (rows 16kq + 4g + q of each tile's samples)
        auto load_x = [&](int kq, f32x4 (&x)[T]) {
#pragma unroll
            for (int t = 0; t < T; ++t) {
                if constexpr (IN == LIN_BUF) {
                    x[t] = valid[t] ? *reinterpret_cast<const f32x4*>(a.in + smp[t] * a.ld_in + 16 * kq + 4 * g)
                                    : f32x4{0.f, 0.f, 0.f, 0.f};
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int f = 16 * kq + 4 * g + q;
                        x[t][q] = (valid[t] && f < a.n_in) ? gather_feature(a, a.feat[f], smp[t]) : 0.f;
                    }
                }
            }
        };
        f32x4 xn[T];
        load_x(0, xn);  // prefetched one k-quad ahead
        // DACT epilogues: tile 0's first σ' arguments are loaded during the last k-quad
        // (the epilogues of all waves otherwise hit HBM in one burst)
        constexpr bool kDact = (EPI == LEPI_DACT || XB) && !MASK;  // σ' rows prefetched
        constexpr int HR = (MT < 8 ? MT : 8) / (T > 2 ? 2 : 1);  // σ' arguments in flight
        const int64_t s0h = valid[0] ? smp[0] : a.batch - 1;
        f32x4 h0[kDact ? HR : 1];
        // MASK (DF_LDENSE_MASK_PF): tile 0's relu-mask words are loaded during the last chunk
        // too, into the registers of the B rows that chunk no longer prefetches
        constexpr bool kMaskPf = MASK && DF_LDENSE_MASK_PF;
        auto mask_words = [&](int64_t s, uint4 (&mq)[4]) {
            const int sl = (int)(s & 31);
            const uint32_t* mb = a.hmask + (s >> 5) * 256 + 16 * ((sl >> 2) & 3) + 4 * g;
#pragma unroll
            for (int w = 0; w < 4; ++w) mq[w] = *reinterpret_cast<const uint4*>(mb + 64 * w);
        };
        uint4 mq0[kMaskPf ? 4 : 1];
        if constexpr (SPLIT && IN == LIN_BUF) {
            f32x4 xn1[T];
            load_x(1, xn1);
            for (int c = 0; c < nchunks; ++c, ++i) {
                const uint8_t* buf = smem;
                if (nchunks > 1) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                    if (i + 1 < total) dma((int)((i + 1) % nchunks), smem + (((i + 1) & 1) ? chunk_bytes : 0));
                    buf = smem + ((i & 1) ? chunk_bytes : 0);
                }
                uni::bf16x8 xp[T][3];
#pragma unroll
                for (int t = 0; t < T; ++t) split8x(xn[t], xn1[t], xp[t][0], xp[t][1], xp[t][2]);
                if (c + 1 < nchunks) {
                    load_x(2 * c + 2, xn);
                    load_x(2 * c + 3, xn1);
                }
                if constexpr (kDact) {
                    if (c + 1 == nchunks) {
#pragma unroll
                        for (int m = 0; m < HR; ++m)
                            h0[m] = *reinterpret_cast<const f32x4*>(a.hprev + s0h * a.ld_h + 4 * g + 16 * m);
                    }
                }
                if constexpr (kMaskPf) {
                    if (c + 1 == nchunks) mask_words(s0h, mq0);
                }
                const uint8_t* wb = buf + lane * 16;
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const uni::bf16x8 w0 = *reinterpret_cast<const uni::bf16x8*>(wb + m * 3072);
                    const uni::bf16x8 w1 = *reinterpret_cast<const uni::bf16x8*>(wb + m * 3072 + 1024);
                    const uni::bf16x8 w2 = *reinterpret_cast<const uni::bf16x8*>(wb + m * 3072 + 2048);
#pragma unroll
                    for (int t = 0; t < T; ++t) {  // small terms first
                        f32x4 v = acc[t][m];
                        v = uni::mfma_bf(w2, xp[t][0], v);
                        v = uni::mfma_bf(w1, xp[t][1], v);
                        v = uni::mfma_bf(w0, xp[t][2], v);
                        v = uni::mfma_bf(w1, xp[t][0], v);
                        v = uni::mfma_bf(w0, xp[t][1], v);
                        acc[t][m] = uni::mfma_bf(w0, xp[t][0], v);
                    }
                }
            }
        } else
        for (int c = 0; c < nchunks; ++c, ++i) {
            const uint8_t* buf = smem;
            if (nchunks > 1) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk i landed (this wave's part)
                __syncthreads();                                     // ... all parts; buffer (i+1)&1 free
                if (i + 1 < total) dma((int)((i + 1) % nchunks), smem + (((i + 1) & 1) ? chunk_bytes : 0));
                buf = smem + ((i & 1) ? chunk_bytes : 0);
            }
            const int kq0 = c * a.chunk_kq;
            const int kq1 = (kq0 + a.chunk_kq < a.nkq) ? kq0 + a.chunk_kq : a.nkq;
            for (int kq = kq0; kq < kq1; ++kq) {
                f32x4 x[T];
#pragma unroll
                for (int t = 0; t < T; ++t) x[t] = xn[t];
                if (kq + 1 < a.nkq) load_x(kq + 1, xn);
                if constexpr (kDact) {
                    if (kq + 1 == a.nkq) {
#pragma unroll
                        for (int m = 0; m < HR; ++m)
                            h0[m] = *reinterpret_cast<const f32x4*>(a.hprev + s0h * a.ld_h + 4 * g + 16 * m);
                    }
                }
                if constexpr (IN == LIN_GATHER) {
#pragma unroll
                    for (int t = 0; t < T; ++t)
                        if (a.xsave && valid[t])
                            *reinterpret_cast<f32x4*>(a.xsave + smp[t] * a.ld_x + 16 * kq + 4 * g) = x[t];
                }
                const uint8_t* wb = buf + (kq - kq0) * MT * 1024 + lane * 16;
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const f32x4 w = lds4(wb + m * 1024);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int t = 0; t < T; ++t) acc[t][m] = mfma4(w[q], x[t][q], acc[t][m]);
                }
            }
        }

        // ---- epilogue: rows 16m + 4g + q of sample smp[t] ----
        if constexpr (EPI == LEPI_DACT || XB) {
#if DF_LDENSE_DIAG == 1  // timing diagnostic (wrong results): δ stored without σ' or x̄
#pragma unroll
            for (int t = 0; t < T; ++t)
                if (valid[t])
#pragma unroll
                    for (int m = 0; m < MT; ++m)
                        *reinterpret_cast<f32x4*>(a.out + smp[t] * a.ld_out + 16 * m + 4 * g) = acc[t][m];
            if (true) continue;
#endif
#pragma unroll
            for (int t = 0; t < T; ++t) {
                // the σ' arguments of the whole tile are loaded at once (a padding
                // sample reads the last row; its δ is zeroed and never stored)
                const int64_t s = valid[t] ? smp[t] : a.batch - 1;
                // XB: the z̄ entries x̄ adds to, read before the δ epilogue (DF_LDENSE_ZV_EARLY: their
                // latency then overlaps it and the x̄ product; z̄ and the δ rows are separate buffers)
                uint32_t zoff[4];  // the columns of features 16m + 4g + q, a byte per q
                float zv[4][4];
                auto load_zv = [&]() {
                    const uint8_t* zcol = w0t_lds + ((SPLIT && a.w0s) ? (a.w0t_nkq / 2) * a.w0t_mt * 3072
                                                                       : a.w0t_mt * a.w0t_nkq * 1024);
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        if (m < a.w0t_mt) {
                            zoff[m] = *reinterpret_cast<const uint32_t*>(zcol + 16 * m + 4 * g);
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const uint32_t c = (zoff[m] >> (8 * q)) & 0xffu;
                                zv[m][q] = a.zbar[s * a.d + (c != 0xffu ? c : 0u)];
                            }
                        }
                    }
                };
                if constexpr (XB && DF_LDENSE_ZV_EARLY) load_zv();
                if constexpr (MASK) {  // relu σ' from the mask of the H0-recomputing split dW1 (no H read)
                    // sample s = 32S + 16tt + 4g' + r: rows 16(4w + mm) + 4g + q in dwords
                    // (S·4 + w)·64 + 16g' + 4g + q, bit 4(2mm + tt) + r (df_ltrain.h LdwArgs::hmask)
                    const int sl = (int)(s & 31);
                    const int sh = 4 * ((sl >> 4) & 1) + (sl & 3);
                    uint4 mq[4];
                    if (kMaskPf && t == 0) {
#pragma unroll
                        for (int w = 0; w < 4; ++w) mq[w] = mq0[kMaskPf ? w : 0];
                    } else {
                        mask_words(s, mq);
                    }
#pragma unroll
                    for (int m = 0; m < MT; ++m) {
                        f32x4 v = acc[t][m];
                        const uint4 u = mq[m >> 2];
                        const int b = 8 * (m & 3) + sh;
                        const uint32_t qb[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = ((qb[q] >> b) & 1u) ? v[q] : 0.f;
                        if (!valid[t]) v = f32x4{0.f, 0.f, 0.f, 0.f};
                        else *reinterpret_cast<f32x4*>(a.out + s * a.ld_out + 16 * m + 4 * g) = v;
                        if constexpr (XB) acc[t][m] = v;  // δ0 → B operand of W0ᵀ
                    }
                } else {
                const float* hrow = a.hprev + s * a.ld_h + 4 * g;
                f32x4 h[HR];
#pragma unroll
                for (int m = 0; m < HR; ++m) h[m] = t == 0 ? h0[m] : *reinterpret_cast<const f32x4*>(hrow + 16 * m);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    f32x4 v = acc[t][m];
                    const f32x4 hm = h[m % HR];
                    if (m + HR < MT) h[m % HR] = *reinterpret_cast<const f32x4*>(hrow + 16 * (m + HR));
                    if (a.dact == DF_ACT_RELU) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = (hm[q] > 0.f) ? v[q] : 0.f;
                    } else if (a.dact != DF_ACT_IDENTITY) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = v[q] * trn::act_grad(a.dact, hm[q]);
                    }
                    if (!valid[t]) v = f32x4{0.f, 0.f, 0.f, 0.f};
                    else *reinterpret_cast<f32x4*>(a.out + s * a.ld_out + 16 * m + 4 * g) = v;
                    if constexpr (XB) acc[t][m] = v;  // δ0 → B operand of W0ᵀ
                }
                }
                if constexpr (XB) {
                    // x̄ = W0ᵀ δ0 (rows = conditioner features, <= 4 tiles) → z̄ of identity dims
                    // The z̄ entries it adds to are read ahead of the product (their latency
                    // overlaps its MFMAs), all loads ahead of all stores: distinct features
                    // of a sample map to distinct state slots (axis_nn).
                    if constexpr (!DF_LDENSE_ZV_EARLY) load_zv();
                    f32x4 xb[4];
#pragma unroll
                    for (int m = 0; m < 4; ++m) xb[m] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (SPLIT && a.w0s) {
                        // bf16x3 split products on bf16 MFMA: δ0's accumulator tiles 2c, 2c+1 are
                        // one B operand (k = 32c + 16(e>>2) + 4g + (e&3), the W1ᵀ planes' order)
#pragma unroll
                        for (int c = 0; c < MT / 2; ++c) {
                            if (2 * c < a.w0t_nkq) {
                                uni::bf16x8 x0, x1, x2;
                                split8x(acc[t][2 * c], acc[t][2 * c + 1], x0, x1, x2);
#pragma unroll
                                for (int m = 0; m < 4; ++m) {
                                    if (m < a.w0t_mt) {
                                        const uint8_t* wp = w0t_lds + (c * a.w0t_mt + m) * 3072 + lane * 16;
                                        const uni::bf16x8 w0 = *reinterpret_cast<const uni::bf16x8*>(wp);
                                        const uni::bf16x8 w1 = *reinterpret_cast<const uni::bf16x8*>(wp + 1024);
                                        const uni::bf16x8 w2 = *reinterpret_cast<const uni::bf16x8*>(wp + 2048);
                                        f32x4 u = xb[m];  // small terms first
                                        u = uni::mfma_bf(w2, x0, u);
                                        u = uni::mfma_bf(w1, x1, u);
                                        u = uni::mfma_bf(w0, x2, u);
                                        u = uni::mfma_bf(w1, x0, u);
                                        u = uni::mfma_bf(w0, x1, u);
                                        xb[m] = uni::mfma_bf(w0, x0, u);
                                    }
                                }
                            }
                        }
                    } else
#pragma unroll
                    for (int kq = 0; kq < MT; ++kq) {
                        if (kq < a.w0t_nkq) {
#pragma unroll
                            for (int m = 0; m < 4; ++m) {
                                if (m < a.w0t_mt) {
                                    const f32x4 w = lds4(w0t_lds + (kq * a.w0t_mt + m) * 1024 + lane * 16);
#pragma unroll
                                    for (int q = 0; q < 4; ++q) xb[m] = mfma4(w[q], acc[t][kq][q], xb[m]);
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int m = 0; m < 4; ++m)
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (m < a.w0t_mt && valid[t]) {
                                const uint32_t c = (zoff[m] >> (8 * q)) & 0xffu;
                                if (c != 0xffu) a.zbar[s * a.d + c] = zv[m][q] + xb[m][q];
                            }
                }
            }
        } else {
#pragma unroll
            for (int t = 0; t < T; ++t) {
                if (!valid[t]) continue;
                const int64_t s = smp[t];
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const int row0 = 16 * m + 4 * g;
                    f32x4 v = acc[t][m];
                    f32x4 pre = v;
                    if constexpr (EPI == LEPI_ACT || EPI == LEPI_COUPLE) {
                        if (a.bias) v = v + *reinterpret_cast<const f32x4*>(a.bias + row0);  // W*x .+ b
                        pre = v;
                        if (a.act != DF_ACT_IDENTITY)
#pragma unroll
                            for (int q = 0; q < 4; ++q) v[q] = impl::act_fn(a.act, v[q]);
                    }
                    if constexpr (EPI == LEPI_ACT) {
                        *reinterpret_cast<f32x4*>(a.out + s * a.ld_out + row0) = v;
                        if (a.dsave) {  // σ'(x) for a pre-activation σ (trn::kDactStored)
                            f32x4 dv;
#pragma unroll
                            for (int q = 0; q < 4; ++q) dv[q] = trn::act_dx(a.act, pre[q], v[q]);
                            *reinterpret_cast<f32x4*>(a.dsave + s * a.ld_out + row0) = dv;
                        }
                    } else if constexpr (EPI == LEPI_COUPLE) {
                        // coupling pullback, rrule(RNVP_backward) src/affine/RNVP.jl:133-139
                        f32x4 dy = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int row = row0 + q;
                            if (row < a.n_af) {
                                const int dim = a.af[row] - a.n;
                                const float zb = a.zbar[s * a.d + dim];
                                float dq;
                                if (a.phase == TR_PHASE_S) {
                                    a.ebuf[s * 32 + row] = expf(-v[q]);
                                    dq = -zb * a.u_out[s * a.d + dim] + a.inv_n;  // s̄ = -z̄_af·z_af - j̄
                                } else {
                                    const bool rnvp = (a.kind == DF_LAYER_RNVP);
                                    const float e = rnvp ? a.ebuf[s * 32 + row] : 1.f;
                                    dq = -zb * e;                                   // t̄ = -z̄_af·exp(-s)
                                    if (rnvp) a.zbar[s * a.d + dim] = zb * e;       // ū_af = z̄_af·exp(-s)
                                }
                                if (a.act != DF_ACT_IDENTITY) dq = dq * trn::act_dx(a.act, pre[q], v[q]);
                                dy[q] = dq;
                            }
                        }
                        *reinterpret_cast<f32x4*>(a.out + s * a.ld_out + row0) = dy;
                    } else {  // LEPI_XBAR: conditioner-input gradient into z̄ of identity dims
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int f = row0 + q;
                            if (f < a.n_in) {
                                const int slot = a.feat[f];
                                if (slot >= a.n && slot < a.n + a.d) a.zbar[s * a.d + (slot - a.n)] += v[q];
                            }
                        }
                    }
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Output Dense + coupling pullback, then δ = (W_outᵀ ȳ) ⊙ σ'(H): H (the last hidden
// activation, kept by the inverse pass) is read once and serves as the B operand of
// the first product and as the σ' argument of the second; ȳ stays in registers as
// the B operand of the second (accumulator layout = B layout).  One 16-sample tile
// per wave per round; both fragment sets resident in LDS.
#ifndef DF_FRONT_DWO
#define DF_FRONT_DWO 1
#endif
// DF_FRONT_DWO (one output tile): the front also accumulates its net's output-Dense dW =
// ȳ·Hᵀ and db = Σ ȳ from the ȳ and H it already holds — the separate narrow dW product
// would read H from HBM a second time.  Per tile: ȳ and each 16-row block of H go through
// a per-wave LDS transpose (trn::t_write / trn::tread: samples onto the MFMA k slots), 4
// f32 MFMAs per block; the 8 waves are summed in LDS in wave order and each workgroup
// writes its partial row (bitwise reproducible, like every other dW).
constexpr int kFrontDwoTS = 16 * kTS;  // floats of one 16-row transpose block
// H blocks moved through LDS per round trip (DF_FRONT_DWO_NB): NB writes, one wait, NB reads
// instead of a wait before and after every block (two lgkmcnt(0) per 16 rows of H)
#ifndef DF_FRONT_DWO_NB
#define DF_FRONT_DWO_NB 4
#endif
constexpr int kDwoNB = DF_FRONT_DWO_NB;
size_t front_dwo_lds_bytes(int ht) {
    const size_t tr = (size_t)kWavesPerBlock * (1 + kDwoNB) * kFrontDwoTS * 4;  // ȳ and H blocks per wave
    const size_t red = (size_t)16 * (16 * ht + 4) * 4 + (size_t)kWavesPerBlock * 256 * 4;  // dW rows + db lanes
    return tr > red ? tr : red;
}

template <int HT, int MTO>
__device__ __forceinline__ void couple_body(const LDenseArgs& a, uint8_t* smem, int bid, int nb) {
    uint8_t* wo = smem;                         // W_out: [kq < HT][m < MTO]
    uint8_t* wt = smem + HT * MTO * 1024;       // W_outᵀ: [kq < MTO][m < HT]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    constexpr bool DWO = (MTO == 1) && DF_FRONT_DWO;
#ifndef DF_FRONT_DWO_PF
#define DF_FRONT_DWO_PF 0
#endif
    constexpr bool HPF = !DWO || DF_FRONT_DWO_PF;  // H of the next tile prefetched
    float* dscr = reinterpret_cast<float*>(smem + 2 * HT * MTO * 1024);  // DWO scratch (front_dwo_lds_bytes)
    float* Ty = dscr + wave * (1 + kDwoNB) * kFrontDwoTS;  // this wave's ȳ block [o][sample] ...
    float* Th = Ty + kFrontDwoTS;                          // ... and kDwoNB H blocks [row][sample]
    f32x4 gwo[DWO ? HT : 1];                    // dW[o = 4g + r][16kq + j]
    float gbo[4] = {0.f, 0.f, 0.f, 0.f};        // Σ ȳ[4g + r] over this lane's samples
#pragma unroll
    for (int kq = 0; kq < (DWO ? HT : 1); ++kq) gwo[kq] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
        const int n1 = a.nkq * MTO * 64, n2 = a.nkq2 * HT * 64;
        for (int q = tid; q < n1; q += kBlockThreads)
            reinterpret_cast<f32x4*>(wo)[q] = reinterpret_cast<const f32x4*>(a.wfrag)[q];
        for (int q = tid; q < n2; q += kBlockThreads)
            reinterpret_cast<f32x4*>(wt)[q] = reinterpret_cast<const f32x4*>(a.w2frag)[q];
    }
    __syncthreads();
    const int64_t ntiles = (a.batch + 15) / 16;
    const bool sph = (a.phase == TR_PHASE_S);
    const bool rnvp = (a.kind == DF_LAYER_RNVP);
    // H of the next tile is loaded while this one is processed (rows of a padding
    // sample read the last sample's; its results are never stored)
    const int64_t tstride = (int64_t)nb * kWavesPerBlock;
    f32x4 hn[HT];
    auto load_h = [&](int64_t tile) {
        int64_t sl = tile * 16 + j;
        sl = sl < a.batch ? sl : a.batch - 1;
#pragma unroll
        for (int kq = 0; kq < HT; ++kq)
            hn[kq] = kq < a.nkq ? *reinterpret_cast<const f32x4*>(a.in + sl * a.ld_in + 16 * kq + 4 * g)
                                : f32x4{0.f, 0.f, 0.f, 0.f};
    };
    // the pullback's operands of rows 16m + 4g + q (transformed dims af[row]): the dims are
    // fixed per lane (hoisted, one byte each; 0xff: no transformed dim), and z̄, u_out (s
    // phases) or exp(−s) (t phases) of the next tile are loaded as soon as this tile's are
    // consumed — no dependent global round trip inside the tile
    uint32_t dimw[MTO];
#pragma unroll
    for (int m = 0; m < MTO; ++m) {
        dimw[m] = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * m + 4 * g + q;
            dimw[m] |= (uint32_t)(row < a.n_af ? a.af[row] - a.n : 0xff) << (8 * q);
        }
    }
    auto dimq = [&](int m, int q) { return (int)((dimw[m] >> (8 * q)) & 0xffu); };
    float zbn[MTO][4], oun[MTO][4];
    auto load_p = [&](int64_t tile) {
        int64_t sl = tile * 16 + j;
        sl = sl < a.batch ? sl : a.batch - 1;
#pragma unroll
        for (int m = 0; m < MTO; ++m)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int dim = dimq(m, q);
                zbn[m][q] = dim != 0xff ? a.zbar[sl * a.d + dim] : 0.f;
                oun[m][q] = dim == 0xff ? 0.f
                            : sph  ? a.u_out[sl * a.d + dim]
                            : rnvp ? a.ebuf[sl * 32 + 16 * m + 4 * g + q]
                                   : 1.f;
            }
    };
    // (MTO = 2: the operands of the tile itself, loaded at its pullback — the prefetch's
    // registers would spill there)
    constexpr bool PFP = (MTO == 1);
    // (DWO: H of the tile loaded at its start — the prefetch's registers hold dW instead)
    if ((int64_t)bid * kWavesPerBlock + wave < ntiles) {
        if (HPF) load_h((int64_t)bid * kWavesPerBlock + wave);
        if (PFP) load_p((int64_t)bid * kWavesPerBlock + wave);
    }
    for (int64_t tile = (int64_t)bid * kWavesPerBlock + wave; tile < ntiles; tile += tstride) {
        const int64_t s = tile * 16 + j;
        const bool valid = s < a.batch;
        f32x4 h[HT];
        if (!HPF) load_h(tile);
#pragma unroll
        for (int kq = 0; kq < HT; ++kq) h[kq] = hn[kq];
        if (HPF && tile + tstride < ntiles) load_h(tile + tstride);
        f32x4 y[MTO];
#pragma unroll
        for (int m = 0; m < MTO; ++m) y[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kq = 0; kq < HT; ++kq) {
            if (kq < a.nkq) {
#pragma unroll
                for (int m = 0; m < MTO; ++m) {
                    const f32x4 w = lds4(wo + (kq * MTO + m) * 1024 + lane * 16);
#pragma unroll
                    for (int q = 0; q < 4; ++q) y[m] = mfma4(w[q], h[kq][q], y[m]);
                }
            }
        }
        // σo(W_out h .+ b), then the coupling pullback (rrule(RNVP_backward) RNVP.jl:133-139)
        if (!PFP) load_p(tile);
        f32x4 dy[MTO];
#pragma unroll
        for (int m = 0; m < MTO; ++m) {
            const int row0 = 16 * m + 4 * g;
            f32x4 v = y[m];
            if (a.bias) v = v + *reinterpret_cast<const f32x4*>(a.bias + row0);
            const f32x4 pre = v;
            if (a.act != DF_ACT_IDENTITY)
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = impl::act_fn(a.act, v[q]);
            dy[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = row0 + q;
                if (valid && row < a.n_af) {
                    const int dim = dimq(m, q);
                    const float zb = zbn[m][q];
                    float dq;
                    if (sph) {
                        a.ebuf[s * 32 + row] = expf(-v[q]);
                        dq = -zb * oun[m][q] + a.inv_n;                 // s̄ = -z̄_af·z_af - j̄
                    } else {
                        const float e = oun[m][q];                     // exp(-s) (RNVP) or 1 (NICE)
                        dq = -zb * e;                                   // t̄ = -z̄_af·exp(-s)
                        if (rnvp) a.zbar[s * a.d + dim] = zb * e;       // ū_af = z̄_af·exp(-s)
                    }
                    if (a.act != DF_ACT_IDENTITY) dq = dq * trn::act_dx(a.act, pre[q], v[q]);
                    dy[m][q] = dq;
                }
            }
            if (valid) *reinterpret_cast<f32x4*>(a.out + s * a.ld_out + row0) = dy[m];
        }
        if (PFP && tile + tstride < ntiles) load_p(tile + tstride);  // this tile's operands consumed
        // δ = (W_outᵀ ȳ) ⊙ σ'(h), one 16-row tile at a time (its product, σ' and store: 4
        // accumulator registers live instead of 4·HT)
        constexpr int MB = 1;
#pragma unroll
        for (int m0 = 0; m0 < HT; m0 += MB) {
            f32x4 acc[MB];
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kq = 0; kq < MTO; ++kq) {
                if (kq < a.nkq2) {
#pragma unroll
                    for (int mb = 0; mb < MB; ++mb) {
                        const f32x4 w = lds4(wt + (kq * HT + m0 + mb) * 1024 + lane * 16);
#pragma unroll
                        for (int q = 0; q < 4; ++q) acc[mb] = mfma4(w[q], dy[kq][q], acc[mb]);
                    }
                }
            }
            if (valid) {
#pragma unroll
                for (int mb = 0; mb < MB; ++mb) {
                    const int m = m0 + mb;
                    f32x4 v = acc[mb];
                    if (a.dact == DF_ACT_RELU) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = (h[m][q] > 0.f) ? v[q] : 0.f;
                    } else if (a.dact != DF_ACT_IDENTITY) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = v[q] * trn::act_grad(a.dact, h[m][q]);
                    }
                    *reinterpret_cast<f32x4*>(a.out2 + s * a.ld_out + 16 * m + 4 * g) = v;
                }
            }
        }
        if constexpr (DWO) {  // dW += ȳ·Hᵀ over the tile's samples (a padding sample's ȳ is 0)
            // every t_write → tread pair ordered by trn::lds_order (lgkmcnt(0) + a memory
            // clobber), the training kernel's convention: the reads must follow the writes
            // and the next rewrite of the transpose rows must follow the reads
            trn::t_write<1>(Ty, dy);
            trn::lds_order();
#pragma unroll
            for (int q = 0; q < 4; ++q) gbo[q] += dy[0][q];
            const f32x4 ya = trn::tread(Ty, j, g);  // ȳ[o = j][samples 4g .. 4g + 3]
#pragma unroll
            for (int k0 = 0; k0 < HT; k0 += kDwoNB) {
                trn::lds_order();  // the previous group's reads returned before its blocks are rewritten
#pragma unroll
                for (int b = 0; b < kDwoNB; ++b) {
                    const int kq = k0 + b;
                    if (kq < HT && kq < a.nkq) {
                        const f32x4 hk[1] = {h[kq < HT ? kq : 0]};
                        trn::t_write<1>(Th + b * kFrontDwoTS, hk);
                    }
                }
                trn::lds_order();
#pragma unroll
                for (int b = 0; b < kDwoNB; ++b) {
                    const int kq = k0 + b;
                    if (kq < HT && kq < a.nkq) {
                        const f32x4 hb = trn::tread(Th + b * kFrontDwoTS, j, g);  // H[16kq + j][samples 4g ..]
#pragma unroll
                        for (int q = 0; q < 4; ++q) gwo[kq < HT ? kq : 0] = mfma4(ya[q], hb[q], gwo[kq < HT ? kq : 0]);
                    }
                }
            }
        }
    }
    if constexpr (DWO) {  // workgroup sum in wave order → this workgroup's partial row
        constexpr int RS = 16 * HT + 4;  // row stride of the dW rows (the two row groups of a b32 half-wave 16 banks apart)
        float* R = dscr;
        float* D = dscr + 16 * RS;  // db lanes [wave][64]
        __syncthreads();
        for (int w = 0; w < kWavesPerBlock; ++w) {
            if (wave == w) {
#pragma unroll
                for (int kq = 0; kq < HT; ++kq)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float* p = R + (4 * g + r) * RS + 16 * kq + j;
                        *p = (w == 0 ? 0.f : *p) + gwo[kq][r];
                    }
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) D[wave * 256 + 64 * q + lane] = gbo[q];
        __syncthreads();
        float* dst = a.dwo_partial + (int64_t)bid * a.dwo_p_total;
        const int mt = a.dwo_m_true, nt = a.dwo_n_true;
        for (int i = tid; i < 16 * 16 * HT; i += kBlockThreads) {
            const int o = i / (16 * HT), col = i - o * (16 * HT);
            if (o < mt && col < nt) dst[a.dwo_w_off + o + mt * col] = R[o * RS + col];
        }
        if (a.dwo_b_off >= 0 && tid < mt) {  // db[o]: lanes (g = o / 4, j) of every wave, q = o % 4
            const int o = tid, q = o & 3, gg = o >> 2;
            float sum = 0.f;
            for (int w = 0; w < kWavesPerBlock; ++w)
                for (int jj = 0; jj < 16; ++jj) sum += D[w * 256 + 64 * q + 16 * gg + jj];
            dst[a.dwo_b_off + o] = sum;
        }
        __syncthreads();  // (the scratch is the next product's staging in a merged launch)
    }
}

template <int HT, int MTO>
__global__ void __launch_bounds__(kBlockThreads, 1) couple_bwd_kernel(LDenseArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    couple_body<HT, MTO>(a, smem, blockIdx.x, gridDim.x);
}

template <int MTO>
void* couple_bwd_ptr_m(int ht) {
    switch (ht) {
        case 1: return reinterpret_cast<void*>(&couple_bwd_kernel<1, MTO>);
        case 2: return reinterpret_cast<void*>(&couple_bwd_kernel<2, MTO>);
        case 4: return reinterpret_cast<void*>(&couple_bwd_kernel<4, MTO>);
        case 8: return reinterpret_cast<void*>(&couple_bwd_kernel<8, MTO>);
        case 16: return reinterpret_cast<void*>(&couple_bwd_kernel<16, MTO>);
        default: return nullptr;
    }
}

void* couple_bwd_ptr(int ht, int mto) { return mto == 2 ? couple_bwd_ptr_m<2>(ht) : couple_bwd_ptr_m<1>(ht); }

// dW = δ · inᵀ and db = Σ δ over this workgroup's contiguous sample range.
// Both operands are staged sample-major in LDS (row stride ≡ 4 mod 8 floats:
// the four lane groups of a half-wave hit disjoint banks), the next stage is
// prefetched into registers while the current one is multiplied.  The 8 waves
// form a wm × (8/wm) grid over the output tiles; each owns bm × bn 16×16
// blocks in registers (k-step q of lane group g uses sample 16u + 4g + q).
// S: samples per staging step (32 for the hidden×hidden dW; 64 for the narrow ones,
// at most 2 × 2 blocks per wave, whose stages are otherwise too short to cover the
// two barriers per step)
template <int S, int BMX, int BNX>  // BMX × BNX: most 16×16 blocks per wave
__device__ __forceinline__ void ldw_body(const LdwArgs& a, float* lsm, int bid, int nblk) {
    const int MA = 16 * a.mta, NB = 16 * a.ntb;
    const int SA = MA + 4, SB = NB + 4;
    float* TA = lsm;
    float* TB = lsm + S * SA;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int wn = kWavesPerBlock / a.wm;
    const int wi = wave % a.wm, wj = wave / a.wm;
    const int m0 = wi * a.bm, n0 = wj * a.bn;  // first row / column tile of this wave
    const int64_t per = (a.batch + nblk - 1) / nblk;
    const int64_t s_begin = (int64_t)bid * per;
    const int64_t s_end = (s_begin + per < a.batch) ? s_begin + per : a.batch;
    (void)wn;

    f32x4 acc[BMX][BNX];
    float db[BMX];
#pragma unroll
    for (int im = 0; im < BMX; ++im) {
        db[im] = 0.f;
#pragma unroll
        for (int in = 0; in < BNX; ++in) acc[im][in] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // staging: thread e of a stage loads one f32x4 (sample e / (rows/4), row quad e % (rows/4))
    const int qa = MA / 4, qb = NB / 4;
    const int na = S * qa, nb = S * qb;
    constexpr int kPre = (S * 256 / 4 + kBlockThreads - 1) / kBlockThreads;  // per operand
    f32x4 pa[kPre], pb[kPre];
    auto fetch = [&](int64_t s0) {
#pragma unroll
        for (int k = 0; k < kPre; ++k) {
            const int e = tid + k * kBlockThreads;
            pa[k] = pb[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (e < na) {
                const int ss = e / qa, rq = e - ss * qa;
                if (s0 + ss < s_end) pa[k] = *reinterpret_cast<const f32x4*>(a.da + (s0 + ss) * a.lda + 4 * rq);
            }
            if (e < nb) {
                const int ss = e / qb, rq = e - ss * qb;
                if (s0 + ss < s_end) pb[k] = *reinterpret_cast<const f32x4*>(a.xb + (s0 + ss) * a.ldb + 4 * rq);
            }
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int k = 0; k < kPre; ++k) {
            const int e = tid + k * kBlockThreads;
            if (e < na) {
                const int ss = e / qa, rq = e - ss * qa;
                *reinterpret_cast<f32x4*>(TA + ss * SA + 4 * rq) = pa[k];
            }
            if (e < nb) {
                const int ss = e / qb, rq = e - ss * qb;
                *reinterpret_cast<f32x4*>(TB + ss * SB + 4 * rq) = pb[k];
            }
        }
    };

    if (s_begin < s_end) fetch(s_begin);
    for (int64_t s0 = s_begin; s0 < s_end; s0 += S) {
        __syncthreads();  // previous stage consumed
        stash();
        __syncthreads();
        if (s0 + S < s_end) fetch(s0 + S);
#pragma unroll
        for (int u = 0; u < S / 16; ++u) {
            const float* ta = TA + (16 * u + 4 * g) * SA + 16 * m0 + j;
            const float* tb = TB + (16 * u + 4 * g) * SB + 16 * n0 + j;
            float fb[BNX][4];
#pragma unroll
            for (int in = 0; in < BNX; ++in)
#pragma unroll
                for (int q = 0; q < 4; ++q) fb[in][q] = (in < a.bn) ? tb[q * SB + 16 * in] : 0.f;
#pragma unroll
            for (int im = 0; im < BMX; ++im) {
                if (im < a.bm) {
                    float fa[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) fa[q] = ta[q * SA + 16 * im];
                    if (wj == 0) db[im] += (fa[0] + fa[1]) + (fa[2] + fa[3]);
#pragma unroll
                    for (int in = 0; in < BNX; ++in)
                        if (in < a.bn)
#pragma unroll
                            for (int q = 0; q < 4; ++q) acc[im][in] = mfma4(fa[q], fb[in][q], acc[im][in]);
                }
            }
        }
    }

    float* dst = a.partial + (int64_t)bid * a.p_total;
#pragma unroll
    for (int im = 0; im < BMX; ++im) {
        if (im >= a.bm || m0 + im >= a.mta) continue;
        const int ma = m0 + im;
#pragma unroll
        for (int in = 0; in < BNX; ++in) {
            if (in >= a.bn || n0 + in >= a.ntb) continue;
            const int nbk = n0 + in;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * ma + 4 * g + r, col = 16 * nbk + j;
                if (row < a.m_true && col < a.n_true) dst[a.w_off + row + (int64_t)a.m_true * col] = acc[im][in][r];
            }
        }
        if (wj == 0) {
            const float v = uni::xgroup_sum(db[im]);
            if (g == 0 && a.b_off >= 0 && 16 * ma + j < a.m_true) dst[a.b_off + 16 * ma + j] = v;
        }
    }
}

// The 256×256 split dW on one wave per SIMD: 4 waves in a 2 × 2 grid of 128 × 128
// quadrants, each wave 8 × 8 blocks of 16×16 (256 accumulator registers: the AGPR half
// of the 512-entry file a lone wave owns).
//
// DF_LDW_DMA (default): per 32-sample step,
//   1. the f32 rows of both operands arrive HBM → LDS by the DMA path (global_load_lds,
//      16 B a lane: one sample row of 256 floats per instruction), issued a whole step
//      ahead (under the previous step's MFMAs) with no registers held for them;
//   2. the workgroup splits every element once: thread (row quad q, sample group sg) of
//      each operand reads its 4 rows × 8 samples (8 ds_read_b128), splits each row's
//      8 samples into three bf16 planes and writes them to LDS as [p][row][32 samples]
//      (64-byte rows; sample-group slot sg ^ ((−row >> 2) & 3), so the fragment
//      ds_read_b128 of the MFMA phase hit 64 distinct banks; the writes are 2-way);
//   3. each wave runs 6 MFMAs per block from the planes (48 ds_read_b128 per 384 MFMAs).
// LDS: 64 KiB f32 stage + 96 KiB planes = the whole 160 KiB; two barriers per step.
// Otherwise: the round-3 form (register prefetch, planes with 80-byte rows).
// db: the f32 sums of each δ row's four 8-sample groups, summed in group order; both
// forms give bitwise the same partial rows for the same grid.
// DF_LDW_DIAG (timing diagnostics, wrong results): 1 = no MFMA phase, 2 = no split phase
#ifndef DF_LDW_DIAG
#define DF_LDW_DIAG 0
#endif
#ifndef DF_LDW_H0_HALVES
#define DF_LDW_H0_HALVES 0
#endif
// compile-time loop: f(std::integral_constant<int, i>) for i < N
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}
#if DF_LDW_DMA
// 16-B slot of 8-sample group sg in plane row `row` (64-B rows): sg XOR bits 1..2 of the row.
// Conflict-free for the MFMA phase's fragment ds_read_b128 (banks (a/4) mod 64, lane groups
// {0–3,12–15,20–27}, ... : 16 distinct (row mod 4, slot) pairs each) and for ds_write_b128 of
// 8 consecutive rows (banks (a/4) mod 32, 8 contiguous lanes: 8 distinct (row mod 2, slot)
// pairs) — MI355X_MICROARCH.md §LDS.  (The round-3 slot sg XOR (−(row >> 2)) & 3 made every
// plane store 2-way: 192 conflict cycles per wave and step, profiles/r05_ldw_lds_conflicts.txt.)
__device__ __forceinline__ int ldw_slot(int row, int sg) { return sg ^ ((row >> 1) & 3); }

// H0R (training with feature snapshots, LdwArgs::feat): the second operand, H0, is not
// read from HBM but recomputed per step from the net's 32-float feature rows with the wide
// SPLIT kernel's first-Dense products (bias, then w2·x0, w1·x1, w0·x2, w1·x0, w0·x1, w0·x0
// onto one accumulator, relu).  The product runs transposed — features as the A operand,
// the W0 fragments (the same bytes) as B — so a lane ends with one H0 row for four
// consecutive samples and writes its bf16x3 planes straight into the B planes (8 bytes
// a plane; no f32 stage, no second split pass).  Wave w computes m-tiles 4w .. 4w + 3 of
// both 16-sample tiles (its 12 W0 fragments and 4 bias values stay in registers), during
// the split phase of the step; the step's feature loads are issued one step ahead.  It
// also writes H0's relu mask for the W1ᵀδ1 epilogue (one ballot per row quad).
template <bool H0R>
__global__ void __launch_bounds__(kLdwSplitThreads, 1) ldw_split_kernel(LdwArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lsm_f[];
    constexpr int PB = 256 * 64;  // bytes per plane
    float* stage = lsm_f;         // [op][32 samples][256]
    uint8_t* TA = reinterpret_cast<uint8_t*>(lsm_f + 2 * 32 * 256);  // δ planes [p][row][64 B]
    uint8_t* TB = TA + 3 * PB;                                       // in planes
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, j = lane & 15;
    const int m0 = 8 * (wave & 1), n0 = 8 * (wave >> 1);
    const int q = lane, sg = wave;  // this thread's staging item of each operand: rows 4q.., samples 8sg..
    const int nblk = gridDim.x;
    // sample range of a workgroup: a multiple of the 32-sample step (steps are aligned blocks
    // of the batch, which the H0R relu-mask layout indexes by)
    // (both instances: the kept-H0 sweep then sums dW1 over the same partition as the
    // H0-free one, which test_h0_free_sweep_bitwise_equals_kept_h0 relies on; the cost is
    // at small batches, where up to half the workgroups of the grid get no step: B = 4096
    // on 256 CUs keeps 128 busy — a few µs per launch at that size)
    const int64_t per = ((a.batch + nblk - 1) / nblk + 31) / 32 * 32;
    const int64_t s_begin = (int64_t)blockIdx.x * per;
    const int64_t s_end = (s_begin + per < a.batch) ? s_begin + per : a.batch;

    f32x4 acc[8][8];
#pragma unroll
    for (int im = 0; im < 8; ++im)
#pragma unroll
        for (int in = 0; in < 8; ++in) acc[im][in] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dbp[4] = {0.f, 0.f, 0.f, 0.f};  // rows q + 64i, sample group sg

    constexpr int NM = H0R ? 4 : 1;  // H0R: m-tiles 4·wave + mm of H0 per wave
    // sample rows s = wave, wave + 4, .. of both operands (64 per step; H0R: δ only, 32); a
    // sample past the workgroup's range is a row of zeros instead
    auto dma = [&](int64_t s0) {
#pragma unroll
        for (int k = 0; k < (H0R ? 8 : 16); ++k) {
            const int r = wave + 4 * k, op = r >> 5, s = r & 31;
            float* dst = stage + (op * 32 + s) * 256;
            if (s0 + s < s_end) {
                const float* src = (op ? a.xb + (s0 + s) * a.ldb : a.da + (s0 + s) * a.lda) + 4 * lane;
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                                 (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
            } else {
                *reinterpret_cast<f32x4*>(dst + 4 * lane) = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    // H0R: this wave's W0 fragments (B operand: lane (g, j) holds W0[16mt + j][8g + e]) and
    // bias values b0[16mt + j], m-tiles mt = 4·wave + mm.  Re-read each step at its top (L2
    // hits: 48 KiB read by every workgroup), their latency under the δ split: held through
    // the MFMA phase they would spill.  The pointers are opaque per step (as loop invariants
    // the loads would be hoisted out of the loop).
    struct W0In {  // (sized for H0R: the other instance never declares one)
        uni::bf16x8 w[4][3];
        float b[4];
    };
    auto h0_wload = [&](W0In& in) {
        const uint8_t* w0p = a.w0s;
        const float* b0p = a.b0;
        asm volatile("" : "+s"(w0p), "+s"(b0p));
#pragma unroll
        for (int mm = 0; mm < NM; ++mm) {
            const int mt = 4 * wave + mm;
#pragma unroll
            for (int p = 0; p < 3; ++p)
                in.w[mm][p] = *reinterpret_cast<const uni::bf16x8*>(w0p + ((mt * 3 + p) << 10) + lane * 16);
            in.b[mm] = b0p[16 * mt + j];
        }
    };
    // H0R: features of samples s0 + 16tt + j (lane group g: 8g .. 8g + 7; past the range:
    // any row, the H0 values are zeroed)
    auto h0_load = [&](int64_t s0, f32x4 (&fr)[2][2]) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            const int64_t s = s0 + 16 * tt + j;
            const int64_t sc = s < s_end ? s : s_begin;
            const f32x4* fp = reinterpret_cast<const f32x4*>(a.feat + sc * 32 + 8 * g);
            fr[tt][0] = fp[0];
            fr[tt][1] = fp[1];
        }
    };
    auto h0_compute = [&](int64_t s0, const f32x4 (&fr)[2][2], const W0In& w0) {
        uni::bf16x8 x[2][3];  // A operand: lane (g, i) holds features 8g + e of sample 16tt + i
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) split8x<DF_LDW_MREM != 0>(fr[tt][0], fr[tt][1], x[tt][0], x[tt][1], x[tt][2]);
        const bool full = s0 + 32 <= s_end;  // (uniform) no sample of the step past the range
        uint32_t mv = 0u;                    // this lane's dword of the wave's relu-mask block
        // (compile-time loops: the mask's v_writelane takes its lane as an inline constant)
        sfor<2>([&](auto mp2c) {
            constexpr int mp2 = decltype(mp2c)::value;
            sfor<2>([&](auto ttc) {
                constexpr int tt = decltype(ttc)::value;
                float hv[8];  // rows 16(4w + 2mp2 + hh) + j, samples 16tt + 4g + r: hv[4hh + r]
                sfor<2>([&](auto hhc) {
                    constexpr int hh = decltype(hhc)::value, mm = 2 * mp2 + hh;
                    f32x4 v = f32x4{w0.b[mm], w0.b[mm], w0.b[mm], w0.b[mm]};
                    v = uni::mfma_bf(x[tt][0], w0.w[mm][2], v);
                    v = uni::mfma_bf(x[tt][1], w0.w[mm][1], v);
                    v = uni::mfma_bf(x[tt][2], w0.w[mm][0], v);
                    v = uni::mfma_bf(x[tt][0], w0.w[mm][1], v);
                    v = uni::mfma_bf(x[tt][1], w0.w[mm][0], v);
                    v = uni::mfma_bf(x[tt][0], w0.w[mm][0], v);
#pragma unroll
                    for (int r = 0; r < 4; ++r) hv[4 * hh + r] = uni::relu_fast(v[r]);
                    if (!full) {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (s0 + 16 * tt + 4 * g + r >= s_end) hv[4 * hh + r] = 0.f;
                    }
                    // relu mask (hmask layout): bit 4(2mm + tt) + r of this lane's dword
#pragma unroll
                    for (int r = 0; r < 4; ++r) mv |= (hv[4 * hh + r] > 0.f ? 1u : 0u) << (4 * (2 * mm + tt) + r);
                });
                uni::bf16x8 p[3];
                split8x<DF_LDW_MREM != 0>(f32x4{hv[0], hv[1], hv[2], hv[3]}, f32x4{hv[4], hv[5], hv[6], hv[7]}, p[0], p[1], p[2]);
                // lane groups g, g ^ 1 hold the two halves (samples 8sg .. +3, +4 .. +7) of
                // the 16-B slots of rows R + j (hh = 0) and R + 16 + j (hh = 1): one
                // v_permlane16_swap per dword gives even groups the whole hh = 0 slot, odd
                // groups the hh = 1 slot, stored by one ds_write_b128 (8 consecutive rows per
                // lane group of the store: conflict-free with ldw_slot)
                const int sgp = 2 * tt + (g >> 1);  // 8-sample group of samples 16tt + 4g ..
                const int row = 16 * (4 * wave + 2 * mp2 + (g & 1)) + j;
                uint8_t* dst = TB + row * 64 + 16 * ldw_slot(row, sgp);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    uint32_t u[4];
                    __builtin_memcpy(u, &p[k], 16);  // dwords 0, 1: hh = 0; 2, 3: hh = 1
                    const auto s0w = __builtin_amdgcn_permlane16_swap(u[0], u[2], false, false);
                    const auto s1w = __builtin_amdgcn_permlane16_swap(u[1], u[3], false, false);
                    // even g: (own hh = 0, g + 1's hh = 0); odd g: (g − 1's hh = 1, own hh = 1)
                    const uint32_t o[4] = {s0w[0], s1w[0], s0w[1], s1w[1]};
                    *reinterpret_cast<uint4*>(dst + k * PB) = uint4{o[0], o[1], o[2], o[3]};
                }
            });
        });
        // the step's 32 samples are one aligned block of the batch (the sample range of a
        // workgroup is a multiple of 32): mask block (s0 / 32, wave), one dword a lane
        a.hmask[((s0 >> 5) * 4 + wave) * 64 + lane] = mv;
    };
    // step 2 for one operand: rows q + 64i, samples 8sg + e (the 8 contiguous lanes of a
    // plane store: 8 consecutive rows; the stage reads: dword reads of 64 consecutive floats,
    // conflict-free).  swz: rows stored with the quad XOR (s & 15) swizzle (unused).
    auto split_item = [&](int op, uint8_t* T, bool db, bool swz) {
        float x[4][8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int s = 8 * sg + e;
                const int r = swz ? ((q + 64 * i) ^ ((s & 15) << 2)) : q + 64 * i;
                x[i][e] = stage[(op * 32 + s) * 256 + r];
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float(&v)[8] = x[i];
            uni::bf16x8 p0, p1, p2;
            split8x<DF_LDW_MREM != 0>(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, p0, p1, p2);
            const int row = q + 64 * i;
            uint8_t* dst = T + row * 64 + 16 * ldw_slot(row, sg);
            *reinterpret_cast<uni::bf16x8*>(dst) = p0;
            *reinterpret_cast<uni::bf16x8*>(dst + PB) = p1;
            *reinterpret_cast<uni::bf16x8*>(dst + 2 * PB) = p2;
            if (db) {
                float sum = dbp[i];
#pragma unroll
                for (int e = 0; e < 8; ++e) sum = sum + v[e];
                dbp[i] = sum;
            }
        }
    };
    auto frag = [&](const uint8_t* T, int row, uni::bf16x8 (&p)[3]) {
        const uint8_t* src = T + row * 64 + 16 * ldw_slot(row, g);
#pragma unroll
        for (int k = 0; k < 3; ++k) p[k] = *reinterpret_cast<const uni::bf16x8*>(src + k * PB);
    };

    [[maybe_unused]] f32x4 fr[2][2];
    if (s_begin < s_end) {
        if constexpr (H0R) h0_load(s_begin, fr);
        dma(s_begin);
    }
    for (int64_t s0 = s_begin; s0 < s_end; s0 += 32) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's rows of the step landed
        __syncthreads();                                     // ... every wave's; the planes are free
#if DF_LDW_DIAG != 2
        if constexpr (H0R) {
            W0In w0;
            h0_wload(w0);  // in flight through the δ split
            split_item(0, TA, true, false);
            h0_compute(s0, fr, w0);
        } else {
            split_item(0, TA, true, false);
            split_item(1, TB, false, false);
        }
#endif
        __syncthreads();                                     // planes written; the stage is free
        const bool more = s0 + 32 < s_end;
        if constexpr (H0R) {
            if (more) h0_load(s0 + 32, fr);  // in flight through the MFMA phase
        }
        if (more) dma(s0 + 32);
#if DF_LDW_DIAG == 1
        continue;
#endif
        // (DF_LDW_H0_HALVES=1, H0R: the column fragments in two halves of 4 — fewer registers
        // through the phase, twice the row-fragment reads; the same products in the same
        // order per accumulator)
        constexpr int NH = (H0R && DF_LDW_H0_HALVES) ? 2 : 1, NI = 8 / NH;
#pragma unroll
        for (int hv = 0; hv < NH; ++hv) {
            uni::bf16x8 xb[NI][3];
#pragma unroll
            for (int in = 0; in < NI; ++in) frag(TB, 16 * (n0 + NI * hv + in) + j, xb[in]);
#pragma unroll
            for (int im = 0; im < 8; ++im) {
                uni::bf16x8 wa[3];
                frag(TA, 16 * (m0 + im) + j, wa);
#pragma unroll
                for (int in = 0; in < NI; ++in) {  // small terms first
                    f32x4 v4 = acc[im][NI * hv + in];
                    v4 = uni::mfma_bf(wa[2], xb[in][0], v4);
                    v4 = uni::mfma_bf(wa[1], xb[in][1], v4);
                    v4 = uni::mfma_bf(wa[0], xb[in][2], v4);
                    v4 = uni::mfma_bf(wa[1], xb[in][0], v4);
                    v4 = uni::mfma_bf(wa[0], xb[in][1], v4);
                    acc[im][NI * hv + in] = uni::mfma_bf(wa[0], xb[in][0], v4);
                }
            }
        }
    }

    float* dst = a.partial + (int64_t)blockIdx.x * a.p_total;
#pragma unroll
    for (int im = 0; im < 8; ++im)
#pragma unroll
        for (int in = 0; in < 8; ++in)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * (m0 + im) + 4 * g + r, col = 16 * (n0 + in) + j;
                if (row < a.m_true && col < a.n_true) dst[a.w_off + row + (int64_t)a.m_true * col] = acc[im][in][r];
            }
    // db[row] = Σ of the row's four sample groups, in group order
    __syncthreads();
    float* dbl = lsm_f;  // [group][row]
#pragma unroll
    for (int i = 0; i < 4; ++i) dbl[256 * sg + q + 64 * i] = dbp[i];
    __syncthreads();
    if (a.b_off >= 0 && tid < a.m_true)
        dst[a.b_off + tid] = ((dbl[tid] + dbl[256 + tid]) + dbl[512 + tid]) + dbl[768 + tid];
}
#else
// Round-3 form: each staging step of 32 samples writes both operands to LDS as planes
// [p][row][sample] (80-byte rows: the 16 rows × 4 lane groups of a ds_read_b128 hit 64
// distinct banks), split once per element; a thread stages row tid of both operands
// (8 strided dword loads per 8 samples, lanes on consecutive rows: coalesced), loaded
// one step ahead, and keeps the f32 sums of its δ row's four sample groups for db.
__global__ void __launch_bounds__(kLdwSplitThreads, 1) ldw_split_kernel(LdwArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lsm_f[];
    uint8_t* lsm = reinterpret_cast<uint8_t*>(lsm_f);
    constexpr int RS = 80;
    constexpr int PB = 256 * RS;
    constexpr int NT = kLdwSplitThreads;
    uint8_t* TA = lsm;
    uint8_t* TB = lsm + 3 * PB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int m0 = 8 * (wave & 1), n0 = 8 * (wave >> 1);
    const int nblk = gridDim.x;
    const int64_t per = (a.batch + nblk - 1) / nblk;
    const int64_t s_begin = (int64_t)blockIdx.x * per;
    const int64_t s_end = (s_begin + per < a.batch) ? s_begin + per : a.batch;

    f32x4 acc[8][8];
#pragma unroll
    for (int im = 0; im < 8; ++im)
#pragma unroll
        for (int in = 0; in < 8; ++in) acc[im][in] = f32x4{0.f, 0.f, 0.f, 0.f};

    // items q = tid + 256k: k < 4 → operand A (row tid, samples 8k..8k+7), k >= 4 → operand B
    float pv[8][8];
    float dbp[4] = {0.f, 0.f, 0.f, 0.f};
    // a whole step of full rows (uniform test): unguarded loads, which the compiler keeps
    // in one basic block; the batch tail and narrower rows take the guarded copy
    const bool full_rows = a.m_true == 256 && a.n_true == 256;
    auto fetch = [&](int64_t s0) {
        if (full_rows && s0 + 32 <= s_end) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float* src = ((k < 4) ? a.da : a.xb) + (s0 + 8 * (k & 3)) * ((k < 4) ? a.lda : a.ldb) + tid;
                const int ld = (k < 4) ? a.lda : a.ldb;
#pragma unroll
                for (int e = 0; e < 8; ++e) pv[k][e] = src[e * ld];
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int sg = k & 3;
            const float* src = (k < 4) ? a.da : a.xb;
            const int ld = (k < 4) ? a.lda : a.ldb;
            const int rmax = (k < 4) ? a.m_true : a.n_true;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int64_t smp = s0 + 8 * sg + e;
                pv[k][e] = (smp < s_end && tid < rmax) ? src[smp * ld + tid] : 0.f;
            }
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uni::bf16x8 x0, x1, x2;
            uni::split8(pv[k], x0, x1, x2);
            uint8_t* base = ((k < 4) ? TA : TB) + tid * RS + 16 * (k & 3);
            *reinterpret_cast<uni::bf16x8*>(base) = x0;
            *reinterpret_cast<uni::bf16x8*>(base + PB) = x1;
            *reinterpret_cast<uni::bf16x8*>(base + 2 * PB) = x2;
            if (k < 4) {
                float sum = dbp[k];
#pragma unroll
                for (int e = 0; e < 8; ++e) sum = sum + pv[k][e];
                dbp[k] = sum;
            }
        }
    };

    if (s_begin < s_end) fetch(s_begin);
    for (int64_t s0 = s_begin; s0 < s_end; s0 += 32) {
        __syncthreads();
        stash();
        __syncthreads();
        if (s0 + 32 < s_end) fetch(s0 + 32);
        uni::bf16x8 xb[8][3];
#pragma unroll
        for (int in = 0; in < 8; ++in)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                xb[in][p] = *reinterpret_cast<const uni::bf16x8*>(TB + p * PB + (16 * (n0 + in) + j) * RS + 16 * g);
#pragma unroll
        for (int im = 0; im < 8; ++im) {
            uni::bf16x8 wa[3];
#pragma unroll
            for (int p = 0; p < 3; ++p)
                wa[p] = *reinterpret_cast<const uni::bf16x8*>(TA + p * PB + (16 * (m0 + im) + j) * RS + 16 * g);
#pragma unroll
            for (int in = 0; in < 8; ++in) {  // small terms first
                f32x4 v = acc[im][in];
                v = uni::mfma_bf(wa[2], xb[in][0], v);
                v = uni::mfma_bf(wa[1], xb[in][1], v);
                v = uni::mfma_bf(wa[0], xb[in][2], v);
                v = uni::mfma_bf(wa[1], xb[in][0], v);
                v = uni::mfma_bf(wa[0], xb[in][1], v);
                acc[im][in] = uni::mfma_bf(wa[0], xb[in][0], v);
            }
        }
    }

    float* dst = a.partial + (int64_t)blockIdx.x * a.p_total;
#pragma unroll
    for (int im = 0; im < 8; ++im)
#pragma unroll
        for (int in = 0; in < 8; ++in)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * (m0 + im) + 4 * g + r, col = 16 * (n0 + in) + j;
                if (row < a.m_true && col < a.n_true) dst[a.w_off + row + (int64_t)a.m_true * col] = acc[im][in][r];
            }
    // db[row] = Σ of the row's four sample groups, in group order
    if (a.b_off >= 0 && tid < a.m_true) dst[a.b_off + tid] = ((dbp[0] + dbp[1]) + dbp[2]) + dbp[3];
}

#endif  // DF_LDW_DMA

void* ldw_split_ptr(bool h0r) {
#if DF_LDW_DMA
    return h0r ? reinterpret_cast<void*>(&ldw_split_kernel<true>) : reinterpret_cast<void*>(&ldw_split_kernel<false>);
#else
    (void)h0r;
    return reinterpret_cast<void*>(&ldw_split_kernel);
#endif
}

template <int S, int BMX, int BNX>
__global__ void __launch_bounds__(kBlockThreads, 1) ldw_kernel(LdwArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    ldw_body<S, BMX, BNX>(a, lsm, blockIdx.x, gridDim.x);
}

// One merged launch of the sweep: the non-split dW products of net i (each workgroup's
// split-K share, as ldw_kernel) and the output-Dense/pullback front of net i+1
// (couple_body, which depends only on z̄ after net i's W1ᵀδ1 kernel).  Even
// workgroups run the front first, odd ones the dW products first, so the fronts and the
// narrow products of the two halves of the CUs interleave.  (The split 256×256 dW is
// its own launch, ldw_split_kernel: one wave per SIMD.)
template <int HT, int MTO>
__global__ void __launch_bounds__(kBlockThreads, 1) sweep_kernel(SweepJob j) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const bool front_first = HT > 0 && j.has_front && (blockIdx.x & 1) == 0;
    if constexpr (HT > 0) {
        if (front_first) {
            couple_body<HT, MTO>(j.front, smem, blockIdx.x, gridDim.x);
            __syncthreads();
        }
    }
    for (int k = 0; k < j.nw; ++k) {
        if (j.ws[k] == 64)
            ldw_body<64, 2, 2>(j.w[k], reinterpret_cast<float*>(smem), blockIdx.x, gridDim.x);
        else
            ldw_body<32, kLdwBM, kLdwBN>(j.w[k], reinterpret_cast<float*>(smem), blockIdx.x, gridDim.x);
        __syncthreads();
    }
    if constexpr (HT > 0) {
        if (j.has_front && !front_first) couple_body<HT, MTO>(j.front, smem, blockIdx.x, gridDim.x);
    }
}

void* sweep_ptr(int ht, int mto) {
    if (ht == 0) return reinterpret_cast<void*>(&sweep_kernel<0, 1>);
    if (ht == 16) return mto == 2 ? reinterpret_cast<void*>(&sweep_kernel<16, 2>)
                                  : reinterpret_cast<void*>(&sweep_kernel<16, 1>);
    if (ht == 8) return mto == 2 ? reinterpret_cast<void*>(&sweep_kernel<8, 2>)
                                 : reinterpret_cast<void*>(&sweep_kernel<8, 1>);
    return nullptr;
}

// One thread per 4 consecutive features of a sample (rows is a multiple of 16): one
// 16-byte store; the index arithmetic is 32-bit (the launcher checks the range).
__global__ void gather_features_kernel(LDenseArgs a, int rows) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t rq = (uint32_t)rows >> 2;
    if (i >= (uint32_t)a.batch * rq) return;
    const uint32_t s = i / rq;
    const int f0 = (int)(i - s * rq) * 4;
    f32x4 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = (f0 + q < a.n_in) ? gather_feature(a, a.feat[f0 + q], s) : 0.f;
    *reinterpret_cast<f32x4*>(a.xsave + (int64_t)s * a.ld_x + f0) = v;
}

template <int MT>
void* ldense_ptr_mt(int in_kind, int epi) {
    if (in_kind == LIN_GATHER) return reinterpret_cast<void*>(&ldense_kernel<MT, LIN_GATHER, LEPI_ACT>);
    switch (epi) {
        case LEPI_ACT: return reinterpret_cast<void*>(&ldense_kernel<MT, LIN_BUF, LEPI_ACT>);
        case LEPI_COUPLE: return reinterpret_cast<void*>(&ldense_kernel<MT, LIN_BUF, LEPI_COUPLE>);
        case LEPI_DACT: return reinterpret_cast<void*>(&ldense_kernel<MT, LIN_BUF, LEPI_DACT>);
        case LEPI_DACT_XBAR: return reinterpret_cast<void*>(&ldense_kernel<MT, LIN_BUF, LEPI_DACT_XBAR>);
        default: return reinterpret_cast<void*>(&ldense_kernel<MT, LIN_BUF, LEPI_XBAR>);
    }
}

void* ldense_ptr(int mt, int in_kind, int epi, bool split = false) {
    if (split) {  // SPLIT instances: the W1ᵀδ1 products of hidden-256 conditioners
        if (mt != 16 || in_kind != LIN_BUF) return nullptr;
        if (epi == LEPI_DACT)
            return reinterpret_cast<void*>(&ldense_kernel<16, LIN_BUF, LEPI_DACT, true, kSplitWaves, kSplitTiles>);
        if (epi == LEPI_DACT_XBAR)
            return reinterpret_cast<void*>(&ldense_kernel<16, LIN_BUF, LEPI_DACT_XBAR, true, kSplitWaves, kSplitTiles>);
        if (epi == LEPI_DACT_XBAR_MASK)
            return reinterpret_cast<void*>(
                &ldense_kernel<16, LIN_BUF, LEPI_DACT_XBAR_MASK, true, kSplitWaves, kSplitTiles>);
        return nullptr;
    }
    switch (mt) {
        case 1: return ldense_ptr_mt<1>(in_kind, epi);
        case 2: return ldense_ptr_mt<2>(in_kind, epi);
        case 4: return ldense_ptr_mt<4>(in_kind, epi);
        case 8: return ldense_ptr_mt<8>(in_kind, epi);
        case 16: return ldense_ptr_mt<16>(in_kind, epi);
        default: return nullptr;
    }
}

}  // namespace

bool ldense_split_supported(int mt, int in_kind, int epi) { return ldense_ptr(mt, in_kind, epi, true) != nullptr; }

hipError_t launch_ldense(int mt, int in_kind, int epi, const LDenseArgs& a, unsigned grid, size_t lds,
                         hipStream_t st) {
    void* k = ldense_ptr(mt, in_kind, epi, a.sfrag != nullptr);
    if (!k) return hipErrorInvalidValue;
    void* args[] = {const_cast<LDenseArgs*>(&a)};
    return hipLaunchKernel(k, dim3(grid), dim3(a.sfrag ? kSplitWaves * 64 : kBlockThreads), args, lds, st);
}

hipError_t ldense_occupancy(int mt, int in_kind, int epi, size_t lds, int* blocks) {
    void* k = ldense_ptr(mt, in_kind, epi);
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, k, kBlockThreads, lds);
}

hipError_t set_ldense_lds_limit(size_t lds) {
    for (int mt : {1, 2, 4, 8, 16}) {
        for (int epi = 0; epi < 5; ++epi) {
            hipError_t e = hipFuncSetAttribute(ldense_ptr(mt, LIN_BUF, epi),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipFuncSetAttribute(ldense_ptr(mt, LIN_GATHER, LEPI_ACT),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    for (int epi : {LEPI_DACT, LEPI_DACT_XBAR, LEPI_DACT_XBAR_MASK}) {
        hipError_t e = hipFuncSetAttribute(ldense_ptr(16, LIN_BUF, epi, true),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<void*>(&ldw_kernel<32, kLdwBM, kLdwBN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldw_lds_bytes());
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute(ldw_split_ptr(false), hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdwSplitLds);
    if (e != hipSuccess) return e;
#if DF_LDW_DMA
    e = hipFuncSetAttribute(ldw_split_ptr(true), hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdwSplitLds);
    if (e != hipSuccess) return e;
#endif
    return hipFuncSetAttribute(reinterpret_cast<void*>(&ldw_kernel<64, 2, 2>), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)ldw_lds_bytes());
}

bool front_dwo(int mto) { return mto == 1 && DF_FRONT_DWO; }
size_t front_dwo_lds(int ht) { return front_dwo_lds_bytes(ht); }

hipError_t launch_couple_bwd(int ht, int mto, const LDenseArgs& a, unsigned grid, size_t lds, hipStream_t st) {
    void* k = couple_bwd_ptr(ht, mto);
    if (!k) return hipErrorInvalidValue;
    void* args[] = {const_cast<LDenseArgs*>(&a)};
    return hipLaunchKernel(k, dim3(grid), dim3(kBlockThreads), args, lds, st);
}

hipError_t set_couple_bwd_lds_limit(size_t lds) {
    for (int ht : {1, 2, 4, 8, 16})
        for (int mto : {1, 2}) {
            hipError_t e = hipFuncSetAttribute(couple_bwd_ptr(ht, mto), hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

hipError_t launch_gather_features(const LDenseArgs& a, int rows, hipStream_t st) {
    const int64_t n = a.batch * (rows / 4);
    if (n <= 0) return hipSuccess;
    if (rows % 4 != 0 || a.ld_x % 4 != 0 || n >= (int64_t(1) << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_features_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, rows);
    return hipGetLastError();
}

// LDS of one staging step: S samples of both operands (row stride rows + 4 floats)
static size_t ldw_stage_bytes(int S, int mta, int ntb) { return (size_t)S * (16 * mta + 4 + 16 * ntb + 4) * 4; }
static int ldw_samples(const LdwArgs& a) {
    return (a.bm <= 2 && a.bn <= 2 && ldw_stage_bytes(64, a.mta, a.ntb) <= kLdwLdsMax) ? 64 : 32;
}
size_t ldw_lds_bytes() { return kLdwLdsMax; }

bool ldw_shape(int mta, int ntb, int* wm, int* bm, int* bn) {
    int best = 1 << 30;
    bool ok = false;
    for (int w : {8, 4, 2, 1}) {
        if (w > kWavesPerBlock) continue;
        const int wn = kWavesPerBlock / w;
        const int m = (mta + w - 1) / w, n = (ntb + wn - 1) / wn;
        if (m <= kLdwBM && n <= kLdwBN && m * n < best) {
            best = m * n;
            *wm = w;
            *bm = m;
            *bn = n;
            ok = true;
        }
    }
    return ok;
}

int ldw_staging_samples(const LdwArgs& a) { return ldw_samples(a); }

bool sweep_supported(int ht, int mto) { return sweep_ptr(ht, mto) != nullptr; }

hipError_t set_sweep_lds_limit(size_t lds) {
    for (int ht : {0, 8, 16})
        for (int mto : {1, 2}) {
            hipError_t e = hipFuncSetAttribute(sweep_ptr(ht, mto), hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

hipError_t launch_sweep(int ht, int mto, const SweepJob& j, unsigned grid, size_t lds, hipStream_t st) {
    void* k = sweep_ptr(j.has_front ? ht : 0, mto);
    if (!k) return hipErrorInvalidValue;
    void* args[] = {const_cast<SweepJob*>(&j)};
    return hipLaunchKernel(k, dim3(grid), dim3(kBlockThreads), args, lds, st);
}

hipError_t launch_ldw(const LdwArgs& a, unsigned grid, hipStream_t st) {
    void* args[] = {const_cast<LdwArgs*>(&a)};
    if (a.split) {
        if (a.mta != 16 || a.ntb != 16) return hipErrorInvalidValue;  // the kernel's fixed 256×256 shape
        const bool h0r = a.feat != nullptr;
        if (h0r && (!DF_LDW_DMA || !a.w0s || !a.b0 || !a.hmask)) return hipErrorInvalidValue;
        return hipLaunchKernel(ldw_split_ptr(h0r), dim3(grid), dim3(kLdwSplitThreads), args, kLdwSplitLds, st);
    }
    const int S = ldw_samples(a);
    void* fn = S == 64 ? reinterpret_cast<void*>(&ldw_kernel<64, 2, 2>)
                       : reinterpret_cast<void*>(&ldw_kernel<32, kLdwBM, kLdwBN>);
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, ldw_stage_bytes(S, a.mta, a.ntb), st);
}

}  // namespace df
