// df_plan.h — device-side chain description shared by the planner (host,
// df_plan.cpp) and the fused kernels (df_kernels.hip).
//
// The planner turns a df_chain_desc (Julia/Flux memory layout) into:
//   * a byte blob holding every Dense of every coupling layer re-laid-out in
//     f32 MFMA (v_mfma_f32_16x16x4_f32) A-fragment order, cut into "stages"
//     that are copied whole into one LDS buffer by all waves of a workgroup;
//   * small uniform descriptor arrays (layers, denses, chunks, stages) that
//     the kernel reads with scalar loads;
//   * an int32 table region (conditioner feature slots, transformed-dim
//     slots) copied to LDS once per workgroup.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "densityflows_hip.h"

namespace df {

constexpr int kWave = 64;
#ifndef DF_BLOCK_WAVES
#define DF_BLOCK_WAVES 8
#endif
#ifndef DF_LDS_TARGET_KB
#define DF_LDS_TARGET_KB 80
#endif
constexpr int kBlockThreads = 64 * DF_BLOCK_WAVES;  // 8 waves per workgroup
constexpr int kWavesPerBlock = kBlockThreads / kWave;
constexpr int kMaxState = 64;        // n + d (conditioner input <= 64 features)
constexpr int kMaxHidden = 256;      // widest Dense (16 MFMA row tiles)
constexpr int kMaxAf = 32;           // transformed dims per coupling layer
constexpr int kMaxLayers = 4096;
constexpr int kStageCap = 24 * 1024;       // LDS weight stage buffer (double-buffered)
constexpr int kSingleStageCap = 64 * 1024; // a whole chain this small lives in one stage
constexpr int kBigStageCap = 64 * 1024;    // stages of wide (>= 128 hidden) generic-kernel chains
constexpr int kStageAlign = 1024;          // one global->LDS DMA wave instruction (64 lanes x 16 B)
constexpr int kMaxTableInts = 4096;  // 16 KiB of int32 tables in LDS
constexpr int kMaxTilesPerWave = 8;          // 16-sample tiles per wave resident in LDS
#ifndef DF_UNI_TT
#define DF_UNI_TT 1
#endif
constexpr int kUniformTileGroup = DF_UNI_TT;  // tiles the specialised kernel evaluates together
#ifndef DF_FAST_TT
#define DF_FAST_TT 2
#endif
constexpr int kFastTileGroup = DF_FAST_TT;    // ... in its FAST variant (fewer live registers per tile)
constexpr int kLdsPerBlockTarget = DF_LDS_TARGET_KB * 1024; // two workgroups per CU

enum : int32_t { IN_STATE = 0, IN_HIDDEN = 1 };

// A contiguous run of k-quads (4 MFMA k-steps each) of one Dense that lives in
// one stage.  Fragment layout inside: [kq - kq_begin][m_tile][lane][4] f32.
struct DevChunk {
    int32_t stage, lds_off, kq_begin, kq_end;
};

struct DevDense {
    int32_t in_kind;     // IN_STATE (conditioner input from the sample state) or IN_HIDDEN
    int32_t ks;          // MFMA k-steps (IN_STATE: ceil(in/4); IN_HIDDEN: 4*kt_in)
    int32_t kt_in;       // IN_HIDDEN: input row tiles of 16
    int32_t mt;          // output row tiles of 16 (MFMA path)
    int32_t out_valu;    // 1: final Dense evaluated as a VALU GEMV (out <= 4)
    int32_t n_out;       // true output width
    int32_t act;         // df_act
    int32_t has_bias;
    int32_t bias_stage, bias_lds;  // bias padded to 16*mt floats (MFMA path)
    int32_t chunk0, n_chunks;
    int32_t w3_stage, w3_lds;      // VALU path: W [n_out][16*kt_in] row-major, then b[4]
    int32_t compact;               // IN_STATE, specialised kernel: [m][r < ks][lane] f32 (no k-quad padding)
    int32_t in_dim;                // true input width
    int32_t w_off, b_off;          // offsets of weight / bias in the flat trainables vector (b_off -1: no bias)
};

struct DevLayer {
    int32_t kind;        // df_layer_kind
    int32_t elem_start;  // first layer (forward order) of its FlowElement
    int32_t elem_end;    // last layer (forward order) of its FlowElement
    int32_t n_af;
    int32_t feat_tab;    // int offset in the table region: [ks*4] state slots
    int32_t af_tab;      // int offset in the table region: [n_af] state slots
    int32_t s_dense0, s_ndense;
    int32_t t_dense0, t_ndense;
    int32_t norm_off;    // NORM: offset in params: x_min[d], x_max[d]
    int32_t out_valu;    // both nets end in a VALU GEMV
    float alpha, beta, ldj_const, pad;
};

// Compact descriptors of the specialised kernel (df_uniform_impl.h): every
// conditioner is Dense(in<=16, H) → nh × Dense(H, H) → Dense(H, out) with
// H = 16·HT, laid out contiguously in ONE stage.
struct UNet {
    int32_t stage;
    int32_t ks;        // first-Dense k-steps (<= 4)
    int32_t nh;        // hidden H×H Denses
    int32_t n_out;
    int32_t off_w0, off_b0;   // byte offsets in the stage
    int32_t off_h, hstride;   // hidden k: W at off_h + k*hstride, bias right after W
    int32_t off_out;          // VALU: W[n_out][H] then b[4]; MFMA: frags then bias
    int32_t act0, acth, act_out;
    int32_t fold0;            // first-Dense bias folded into k-slot 4·ks−1 (state column n+d+3 holds 1)
};

struct ULayer {
    int32_t kind, elem_start, elem_end, n_af;
    int32_t feat_tab, af_tab, norm_off, pad0;
    float alpha, beta, ldj_const, pad1;
    UNet s, t;
};

// Wide-net kernel (df_wide_impl.h): every conditioner is Dense(in <= 64, 256) →
// Dense(256, 256) → Dense(256, out <= 32).  Its weights live in their own blob of
// fixed 32 KiB stages: first Dense (2 k-quads × 16 m-tiles per stage), 8 stages of
// the hidden Dense, one stage of the output Dense ([kq < 16][m < mto]).
constexpr int kWideStageBytes = 32 * 1024;
#ifndef DF_WIDE_NB
#define DF_WIDE_NB 2
#endif
constexpr int kWideBufs = DF_WIDE_NB;   // LDS stage ring: the DMA runs kWideBufs − 1 stages ahead
constexpr int kWideWaves = 4;     // one wave per SIMD (512 registers each)
constexpr int kWideT = 2;         // 16-sample tiles per wave held in registers (3 spills)
#ifndef DF_WSPLIT_HALF
#define DF_WSPLIT_HALF 0
#endif
// SPLIT stages: half a 32-input chunk (8 m-tiles × 3 planes, 24 KiB) in a 4-slot ring
// (the DMA three stages ahead), or (DF_WSPLIT_HALF=0) a whole chunk in a 2-slot ring
constexpr int kWideSplitHalves = DF_WSPLIT_HALF ? 2 : 1;
constexpr int kWideSplitStageBytes = 48 * 1024 / kWideSplitHalves;
constexpr int kWideSplitBufs = DF_WSPLIT_HALF ? 4 : 2;

struct WNet {
    int32_t stage0;   // first stage id (wide blob)
    int32_t nst0;     // stages of the first Dense (1 or 2; SPLIT: chunks × kWideSplitHalves)
    int32_t nso;      // SPLIT: stages of the output Dense (1, or 2 when half stages split mto = 2)
    int32_t ks;       // first-Dense k-steps (ceil(in/4))
    int32_t n_out, mto;
    int32_t act0, act1, act_out;
    int32_t b0, b1, bo;  // float offsets of the (padded) biases in wbias, -1: none
};

struct WLayer {
    int32_t kind, elem_start, elem_end, n_af;
    int32_t feat_tab, af_tab, norm_off, pad0;
    float alpha, beta, ldj_const, pad1;
    WNet s, t;
};

struct DevStage {
    int64_t src_off;     // byte offset in the blob
    int32_t bytes;       // multiple of 16
    int32_t pad;
};

// bf16x3 split of an f32 value (the SPLIT variant of the FAST kernel,
// df_uniform_impl.h): w = p0 + p1 + p2 exactly for every finite w away from the
// bf16 overflow edge, each plane rounded to nearest-even from the remainder of
// the previous ones (8 + 8 + 8 significand bits).  Host packing and the device
// repack kernel use this same integer routine; the kernels split activations
// with v_cvt_pk_bf16_f32, which rounds the same way.
#if defined(__HIPCC__)
#define DF_HD __host__ __device__
#else
#define DF_HD
#endif
DF_HD inline uint16_t bf16_rne_bits(float f) {
    const uint32_t u = __builtin_bit_cast(uint32_t, f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // NaN stays NaN
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
DF_HD inline float bf16_bits_to_f32(uint16_t h) { return __builtin_bit_cast(float, (uint32_t)h << 16); }
DF_HD inline uint16_t bf16_split_plane(float w, int plane) {
    const uint16_t h0 = bf16_rne_bits(w);
    if (plane == 0) return h0;
    const float r = w - bf16_bits_to_f32(h0);
    const uint16_t h1 = bf16_rne_bits(r);
    if (plane == 1) return h1;
    return bf16_rne_bits(r - bf16_bits_to_f32(h1));
}
// SPLIT stage layout of one FAST net (H = 16·HT, HT = 2 or 4), byte offsets from
// the net's start:
//   first Dense  [m < HT][lane][8 bf16]: lane (g, i) holds W[16m+i, g] as the
//                product slots (w0, w0, w1, w0, w1, w2, 0, 0) (g = 3: the folded bias)
//   hidden Dense [c < HT/2][m < HT][plane < 3][lane][8 bf16]: lane (g, i) holds
//                plane p of W1[16m+i, 32c + 16(e>>2) + 4g + (e&3)], e < 8
//   hidden bias  f32 [16·HT]
//   output Dense f32 [n_out][16·HT] then b[4] (VALU GEMV, as in the f32 layout)
constexpr int kSplitFirstBytes(int ht) { return ht * 1024; }
constexpr int kSplitHiddenBytes(int ht) { return (ht / 2) * ht * 3 * 1024; }

struct Plan {
    int d = 0, n = 0, n_layers = 0;
    int stride = 0;          // floats per sample row of the LDS state tile
    int ht = 0;              // kernel variant: max row tiles (1,2,4,8,16)
    int tiles = 0;           // 16-sample tiles per wave resident in LDS
    int outv = 0;            // kernel variant: final Dense as VALU GEMV (<= 4 outputs)
    int uniform = 0;         // every layer fits the specialised kernel (ulayers valid)
    int relu_only = 0;       // specialised kernel variant: hidden σ = relu, output σ = identity
    int tile_group = 1;      // tiles per wave evaluated together (specialised kernel: 1, FAST: 2)
    int fast = 0;            // specialised kernel variant: relu_only, n_sublayers = 2, every first Dense one k-step with its bias folded
    std::vector<ULayer> ulayers;
    int samples_per_block = 0;
    int stage_max = 0;       // largest stage (bytes, multiple of kStageAlign)
    std::vector<int32_t> sched_fwd;  // stage ids in the order a forward pass needs them
    std::vector<int32_t> sched_bwd;  // ... and a backward (inverse) pass
    std::vector<DevLayer> layers;
    std::vector<DevDense> denses;
    std::vector<DevChunk> chunks;
    std::vector<DevStage> stages;
    std::vector<uint8_t> blob;
    std::vector<int32_t> tables;
    std::vector<float> params;
    int64_t n_params = 0;
    // Flux.trainables order (src/affine/RNVP.jl:51, NICE.jl:38, Blocks.jl:77): per
    // coupling layer s_net then t_net, per Dense weight (out×in column-major) then bias.
    std::vector<float> trainables;
    // blob float index ← trainables index, for every blob float that holds a parameter
    std::vector<int32_t> pack_dst, pack_src;
    // wide-net kernel (empty unless every conditioner has the wide default shape)
    int wide = 0;
    std::vector<WLayer> wlayers;
    std::vector<DevStage> wstages;
    std::vector<uint8_t> wblob;
    std::vector<float> wbias;
    std::vector<int32_t> wsched_fwd, wsched_bwd;
    std::vector<int32_t> wpack_dst, wpack_src;   // wblob float index ← trainables index
    std::vector<int32_t> wbias_dst, wbias_src;   // wbias index ← trainables index
    // SPLIT variant of the FAST kernel: the conditioner GEMMs on bf16 MFMA with
    // both operands split in three bf16 planes (6 products, f32 accumulation);
    // its own blob of one-net stages, schedules and descriptors.
    int split = 0;
    int stiles = 0;              // resident 16-sample tiles per wave with the split stages
    int sstage_max = 0;
    std::vector<ULayer> sulayers;
    std::vector<DevStage> sstages;
    std::vector<uint8_t> sblob;
    std::vector<int32_t> ssched_fwd, ssched_bwd;
    // sblob byte offset ← trainables index·4 + plane (plane 3: the f32 value itself)
    std::vector<int32_t> spack_dst, spack_src;
    // SPLIT variant of the wide kernel (plan.wide): first, hidden and output Dense
    // as bf16x3 products; stages of up to kWideSplitStageBytes ([m][plane][lane][8]
    // per 32-input chunk), WLayer::pad0 = the layer's split feature table (32·nst0
    // slots); biases stay in wbias.
    int wsplit = 0;
    std::vector<WLayer> wslayers;
    std::vector<DevStage> wsstages;
    std::vector<uint8_t> wsblob;
    std::vector<int32_t> wssched_fwd, wssched_bwd;
    std::vector<int32_t> wspack_dst, wspack_src;  // wsblob byte offset ← trainables index·4 + plane
    std::vector<int32_t> wstables;                // tables + the split feature tables (wide SPLIT launches)
    double flops_per_sample = 0.0;
    double split_flops_per_sample = 0.0;  // the part of flops_per_sample the SPLIT kernel runs on bf16 MFMA
};

// Returns DF_OK or a df_status; *err receives a message mirroring the
// reference's exception text where one exists.
// exact: plan the exact-f32 kernels only (no SPLIT blobs); -1 = from DF_F32_EXACT
int build_plan(const df_chain_desc* desc, Plan* out, std::string* err, int exact = -1);

// Workgroup LDS bytes for a plan (stage buffers + tables + state tile).
size_t plan_lds_bytes(const Plan& p);
// The NormalizationLayer bounds (`params`) are copied into LDS next to the index tables
// only by the specialised kernel's one-pass copy-in (df_uniform_impl.h fast_copy, which
// needs n_par <= kBlockThreads); every other plan keeps them in HBM.
inline bool params_in_lds(const Plan& p) { return p.uniform && p.params.size() <= (size_t)kBlockThreads; }
// int32 words of the table area: the index tables, then (params_in_lds) the bounds
inline int table_lds_ints(const Plan& p) { return (int)(p.tables.size() + (params_in_lds(p) ? p.params.size() : 0)); }
// LDS bytes of the table area
inline int table_lds_bytes(const Plan& p) { return (table_lds_ints(p) * 4 + 15) / 16 * 16; }

}  // namespace df
