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
constexpr int kBlockThreads = 512;   // 8 waves per workgroup
constexpr int kWavesPerBlock = kBlockThreads / kWave;
constexpr int kMaxState = 64;        // n + d (conditioner input <= 64 features)
constexpr int kMaxHidden = 256;      // widest Dense (16 MFMA row tiles)
constexpr int kMaxAf = 32;           // transformed dims per coupling layer
constexpr int kMaxLayers = 4096;
constexpr int kStageCap = 48 * 1024; // bytes of the LDS weight stage buffer
constexpr int kMaxTableInts = 4096;  // 16 KiB of int32 tables in LDS
#ifndef DF_TILES_SMALL
#define DF_TILES_SMALL 1
#endif
constexpr int kTilesSmall = DF_TILES_SMALL;  // sample tiles per wave for hidden <= 64

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
    int32_t pad0, pad1;
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

struct DevStage {
    int64_t src_off;     // byte offset in the blob
    int32_t bytes;       // multiple of 16
    int32_t pad;
};

struct Plan {
    int d = 0, n = 0, n_layers = 0;
    int stride = 0;          // floats per sample row of the LDS state tile
    int ht = 0;              // kernel variant: max row tiles (1,2,4,8,16)
    int tiles = 0;           // 16-sample MFMA column tiles per wave
    int outv = 0;            // kernel variant: final Dense as VALU GEMV (<= 4 outputs)
    int samples_per_block = 0;
    int stage_max = 0;       // largest stage (bytes)
    std::vector<DevLayer> layers;
    std::vector<DevDense> denses;
    std::vector<DevChunk> chunks;
    std::vector<DevStage> stages;
    std::vector<uint8_t> blob;
    std::vector<int32_t> tables;
    std::vector<float> params;
    int64_t n_params = 0;
    double flops_per_sample = 0.0;
};

// Returns DF_OK or a df_status; *err receives a message mirroring the
// reference's exception text where one exists.
int build_plan(const df_chain_desc* desc, Plan* out, std::string* err);

// Workgroup LDS bytes for a plan (stage buffer + tables + state tile).
size_t plan_lds_bytes(const Plan& p);

}  // namespace df
