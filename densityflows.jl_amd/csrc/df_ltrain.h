// df_ltrain.h — layer-wise training path for conditioners the fused per-net
// kernel (df_train_impl.h) cannot hold in registers (hidden width > 64, more
// than one hidden Dense, > 4 transformed dims; BASELINE config 5: d = 32,
// hidden 256).
//
// Per conditioner net, every Dense becomes one MFMA GEMM over the whole batch
// with a fused epilogue; activations live in HBM in the sample-major layout
// (Julia's (h, B) column-major: sample j's h values contiguous), which is
// exactly the register layout of an MFMA accumulator tile, so loads and stores
// are 16-byte vectors:
//   forward   H0 = σ0(W0 x + b0) (x gathered from vcat(θ, u)[axis_nn], kept),
//             Hk = σk(Wk Hk-1 + bk),  Y = σo(Wo H + bo)
//             → coupling pullback in the epilogue → ȳ  (s̄ / t̄, ū_af)
//   backward  δ = (Wᵀ ȳ) ⊙ σ'(H) per Dense, x̄ = W0ᵀ δ0 → z̄ of identity dims
//   weights   dW = δ · inᵀ, db = Σ δ: split-K over samples, one partial per
//             workgroup (fixed-order reduction afterwards, as the fused path).
// Weight fragments (W and Wᵀ, [kq][m][lane][4]) are streamed through two LDS
// chunk buffers shared by the 8 waves of a workgroup.
#pragma once

#include <hip/hip_runtime.h>

#include "df_plan.h"

namespace df {

enum : int { LIN_BUF = 0, LIN_GATHER = 1 };
enum : int { LEPI_ACT = 0, LEPI_COUPLE = 1, LEPI_DACT = 2, LEPI_XBAR = 3, LEPI_DACT_XBAR = 4,
             LEPI_DACT_XBAR_MASK = 5 };  // (5: SPLIT only, σ' from LDenseArgs::hmask)

constexpr int kLChunkBytes = 32 * 1024;  // weight chunk (LDS, double-buffered)
#ifndef DF_LTILES
#define DF_LTILES 2
#endif
constexpr int kLTiles = DF_LTILES;       // 16-sample tiles per wave per round
#ifndef DF_LDENSE_SPLIT_1W
#define DF_LDENSE_SPLIT_1W 0
#endif
// SPLIT (hidden-256 W1ᵀδ1) instances: waves per workgroup × tiles per wave (samples per
// workgroup round = kWavesPerBlock · kLTiles either way)
constexpr int kSplitWaves = DF_LDENSE_SPLIT_1W ? 4 : kWavesPerBlock;
constexpr int kSplitTiles = DF_LDENSE_SPLIT_1W ? 4 : kLTiles;
constexpr size_t kLdwLdsMax = 80 * 1024; // dW staging LDS (32 or 64 samples per step)
#ifndef DF_LDW_DMA
#define DF_LDW_DMA 1
#endif
#if DF_LDW_DMA  // SPLIT dW: f32 stage of both operands (32 sample rows) + their bf16x3 planes
constexpr size_t kLdwSplitLds = 2 * 32 * 256 * 4 + 2 * 3 * 256 * 64;
#else           // SPLIT dW: both operands' planes, [p][row][32 samples + pad]
constexpr size_t kLdwSplitLds = 2 * 3 * 256 * 80;
#endif
constexpr int kLdwSplitThreads = 256;              // SPLIT dW kernel: one wave per SIMD
constexpr int kLdwBM = 8;                // per-wave output blocks (16×16): up to 8 row tiles
constexpr int kLdwBN = 4;                //   × 4 column tiles (128 accumulator registers)

struct LDenseArgs {
    const uint8_t* wfrag;   // fragments [kq][m][lane][4] of A (M = 16·MT rows)
    const uint8_t* sfrag;   // or (SPLIT, W1ᵀδ1 of hidden-256 nets) bf16x3 planes [c][m][p][lane][8], else nullptr
    const float* bias;      // 16·MT floats or nullptr
    int nkq, chunk_kq;
    int act;                // LEPI_ACT / LEPI_COUPLE: σ of this Dense
    // B operand
    const float* in;        // LIN_BUF: [B][ld_in]
    int ld_in;
    const float* theta;     // LIN_GATHER: vcat(θ, u)[axis_nn] features
    const float* tmin;
    const float* tmax;
    const float* u_in;
    const int32_t* feat;    // feature → state slot (n + d: zero)
    int n_in;               // true conditioner input width (gather / xbar)
    float* xsave;           // LIN_GATHER: gathered features stored [B][ld_x] (may be nullptr)
    int ld_x;
    // epilogue
    float* out;             // [B][ld_out]
    int ld_out;
    float* dsave;           // LEPI_ACT: σ'(pre-activation) stored [B][ld_out] (nets with a
                            // softplus / logcosh / swish σ), or nullptr
    const float* hprev;     // LEPI_DACT: σ'(hprev) with activation dact
    int ld_h, dact;
    float* zbar;            // LEPI_COUPLE / LEPI_XBAR
    const float* u_out;
    float* ebuf;            // [B][32] exp(-s)
    const int32_t* af;
    int n_af, phase, kind;
    float inv_n;
    int64_t batch;
    int d, n;
    // LEPI_DACT_XBAR: x̄ = W0ᵀ δ0 right after δ0 (fragments resident in LDS)
    const uint8_t* w0t;
    int w0t_mt, w0t_nkq;
    const uint8_t* w0s;     // SPLIT instances: W0ᵀ as bf16x3 planes [c][m][p][lane][8] (x̄ on bf16 MFMA), or nullptr
    const uint32_t* hmask;  // LEPI_DACT(_XBAR), relu: σ'(H) from the relu mask of the H0-recomputing split
                            // dW1 (LdwArgs::hmask), else hprev
    // couple_bwd_kernel: second product W_outᵀ ȳ (fragments [kq][m][lane][4], m < 16·HT rows)
    const uint8_t* w2frag;
    int nkq2;
    float* out2;            // δ of the last hidden Dense [B][ld_out]
    // couple_bwd (one output tile, DF_FRONT_DWO): the output Dense's dW = ȳ·Hᵀ and db = Σ ȳ,
    // accumulated by the front from the H and ȳ it holds and written as the workgroup's
    // partial row (layout of ldw: w_off + o + m_true·col, b_off + o)
    float* dwo_partial;
    int64_t dwo_p_total;
    int dwo_w_off, dwo_b_off, dwo_m_true, dwo_n_true;
};

struct LdwArgs {
    const float* da;        // δ  [B][lda] (rows = Dense outputs)
    int lda, m_true;
    const float* xb;        // in [B][ldb] (rows = Dense inputs)
    int ldb, n_true;
    int mta, ntb;           // 16-row tiles of each operand
    int wm, bm, bn;         // waves along M (8/wm along N); blocks per wave bm × bn
    float* partial;         // [workgroup][p_total]
    int64_t p_total;
    int w_off, b_off;       // trainables offsets (b_off -1: no bias)
    int64_t batch;
    int split;              // 1: bf16x3 split products (ldw_split_kernel, its own launch; mta = ntb = 16)
    // split dW1 with H0 recomputed (xb unused): H0 = relu(b0 + W0·f) with the wide SPLIT
    // kernel's first-Dense arithmetic (bitwise its H0), f the net's features [B][32]
    // (ChainArgs::fsave), W0 the first-Dense stage [m < 16][p][lane][8] of the wide split
    // blob; the kernel also writes H0's relu mask for the W1ᵀδ1 epilogue
    const float* feat;
    const uint8_t* w0s;
    const float* b0;
    // relu mask of H0, blocks of 256 dwords per aligned 32-sample step S (= s >> 5): block S,
    // dword (S·4 + w)·64 + 16g' + j, bit 4(2mm + tt) + r ↔ H0 row 16(4w + mm) + j > 0 of
    // sample 32S + 16tt + 4g' + r (the lane (g', j) of wave w that computed it)
    uint32_t* hmask;
};

// One merged launch: up to three non-split dW products (ldw) of net i and, optionally, the
// couple_bwd front of net i+1 (sweep_kernel, df_ltrain.hip).
struct SweepJob {
    LdwArgs w[3];
    int ws[3];              // staging samples of each product (32 or 64, ldw_staging_samples)
    int nw;
    LDenseArgs front;       // couple_bwd arguments of the next net
    int has_front;
};

hipError_t launch_ldense(int mt, int in_kind, int epi, const LDenseArgs& a, unsigned grid, size_t lds,
                         hipStream_t st);
hipError_t ldense_occupancy(int mt, int in_kind, int epi, size_t lds, int* blocks);
// a SPLIT instance exists (LIN_BUF, 16 row tiles, δ epilogues)
bool ldense_split_supported(int mt, int in_kind, int epi);
hipError_t set_ldense_lds_limit(size_t lds);
hipError_t launch_ldw(const LdwArgs& a, unsigned grid, hipStream_t st);
// Output Dense + coupling pullback → ȳ, then δ = (W_outᵀ ȳ) ⊙ σ'(H) in one pass over H
// (ht: 16-row tiles of H, mto: output tiles <= 2).  LDS: both fragment sets.
hipError_t launch_couple_bwd(int ht, int mto, const LDenseArgs& a, unsigned grid, size_t lds, hipStream_t st);
// the front computes its net's output-Dense dW / db (mto 1, DF_FRONT_DWO); the extra LDS it
// needs beyond its fragments, and whether it does
bool front_dwo(int mto);
size_t front_dwo_lds(int ht);
hipError_t set_couple_bwd_lds_limit(size_t lds);
// conditioner input vcat(θ, u)[axis_nn] → xsave [B][ld_x] (rows >= n_in zero), for dW0
hipError_t launch_gather_features(const LDenseArgs& a, int rows, hipStream_t st);
size_t ldw_lds_bytes();
int ldw_staging_samples(const LdwArgs& a);
// sweep_kernel instances exist for fronts of hidden width 128 / 256 (ht 8 / 16), mto 1 / 2
bool sweep_supported(int ht, int mto);
hipError_t set_sweep_lds_limit(size_t lds);
hipError_t launch_sweep(int ht, int mto, const SweepJob& j, unsigned grid, size_t lds, hipStream_t st);
// wave grid and per-wave blocks for a dW of mta × ntb tiles (host helper)
bool ldw_shape(int mta, int ntb, int* wm, int* bm, int* bn);

}  // namespace df
