// df_train.h — launch interface of the training path (reverse sweep of the
// NLL through the inverse pass, Adam, weight repacking).
//
// One training step (src/Flows.jl:396-414: Flux.gradient of
// loss(backward(model, x, θ)) then Optimisers.update!):
//   1. inverse pass on the specialised kernel, keeping every layer's output
//      U[li] ([layer][sample][d], U[0] = z) and the Σ logpdf partials;
//   2. z̄ = z / N (∂loss/∂z for loss = -mean(logpdf(MvNormal(0,I), z) + ldj));
//   3. layers in chain order li = 0..L-1 (reverse of the inverse pass): one
//      train_net_kernel launch per conditioner (s-net, then t-net), which
//      recomputes the net on U[li+1], applies the coupling pullback
//      (rrule(RNVP_backward) src/affine/RNVP.jl:119-143, NICE.jl:102-111),
//      back-propagates through the Dense chain on MFMA, accumulates dW / db per
//      workgroup in registers and updates z̄ in place; NormalizationLayer
//      scales z̄ element-wise;
//   4. a fixed-order reduction of the per-workgroup partials → ∇ (flat,
//      Flux.trainables order); [multi-GPU: the caller all-reduces ∇ here];
//   5. Adam (Optimisers.jl) on the flat parameters, then the packed weight
//      blobs are regathered from them on device.
#pragma once

#include <hip/hip_runtime.h>

#include "df_plan.h"

namespace df {

#ifndef DF_TRAIN_WAVES
#define DF_TRAIN_WAVES 8
#endif
constexpr int kTrainWaves = DF_TRAIN_WAVES;     // waves per workgroup of the fused net kernel
constexpr int kTrainThreads = 64 * kTrainWaves;
// 16-sample tiles one wave of a SPLIT instance carries through the sweep together: with
// 2, a workgroup is kTrainWaves / 2 waves (one per SIMD, VGPRs + AGPRs = 512 per lane)
// and each wave interleaves two independent tiles (df_train_impl.h).  The per-SIMD tile
// count, the LDS transpose area and the tiles per workgroup pass are unchanged.
#ifndef DF_TRAIN_TT
#define DF_TRAIN_TT 1
#endif
constexpr int kTrainSplitTT = DF_TRAIN_TT;
static_assert(kTrainWaves % kTrainSplitTT == 0, "tiles per wave must divide the workgroup's tile count");
constexpr int train_threads(bool split) { return split ? kTrainThreads / kTrainSplitTT : kTrainThreads; }
// Per-wave transpose buffers [row][16 samples] (df_train_impl.h): rows of 20 floats (row
// R and R + 4 of a ds_write_b32 half-wave hit disjoint bank halves) and, with
// DF_TRAIN_SWZ, the 4-float column quads XOR-swizzled by row (trn::rswz: Gray bit of
// (R >> 2) & 3 ^ bit 4 of R) so both b128 fragment read shapes are bank-conflict free too.
#ifndef DF_TRAIN_SWZ
#define DF_TRAIN_SWZ 1
#endif
constexpr int kTS = 20;  // row stride (floats)

namespace trn {
// Activation modes of the training kernels: σ' from the output alone, relu-only,
// or σ' of softplus / logcosh / swish, which needs the pre-activation.
enum { AM_Y = 0, AM_RELU = 1, AM_PRE = 2 };

// σ' applied by the layer-wise δ kernels when the factor was stored at recompute
// time (nets with a pre-activation σ): hprev then holds σ'(x) itself.
constexpr int kDactStored = 64;
}  // namespace trn

// One conditioner net of the specialised shape, as the training kernel sees it.
struct GNet {
    UNet u;                  // forward fragments (offsets rebased to the net's own LDS copy)
    int32_t n_in;            // conditioner inputs (|axis_nn|)
    int32_t h_true;          // hidden width
    int32_t off_w0t;         // transposed region: W0ᵀ fragments [kq < HT][lane][4]
    int32_t off_ht;          // transposed region: W_hᵀ fragments [kq][m][lane][4]
    int32_t fwd_bytes;       // forward region bytes (16-B multiple)
    int32_t t_bytes;         // transposed region bytes
    int64_t fwd_src;         // byte offset of the forward region in the chain blob
    int64_t t_src;           // byte offset of the transposed region in the training blob
    int32_t p_begin, p_count;          // the net's contiguous slice of the trainables
    int32_t w_off[3], b_off[3];        // first Dense, hidden Dense, output Dense (b_off -1: no bias)
    // SPLIT (chain plan.split, hidden 32/64, relu): the recompute runs on the net's
    // region of the chain's SPLIT blob (bitwise the inverse pass), W1ᵀδ and dW1 on
    // bf16x3 products; W1ᵀ planes [c][m][p][lane][8] in the trainer's split blob
    int32_t split;
    UNet su;                 // SPLIT forward region offsets (rebased to the net's LDS copy)
    int32_t sfwd_bytes;
    int64_t sfwd_src;        // byte offset of the net's region in the chain's SPLIT blob
    int32_t st_bytes;
    int64_t st_src;          // byte offset of its W1ᵀ planes in the trainer's split blob
};

enum : int { TR_PHASE_S = 0, TR_PHASE_T = 1 };

struct TrainArgs {
    const float* u_in;       // U[li+1]: the layer's input in the inverse pass
    const float* u_out;      // U[li]:   its output
    const float* theta;
    const float* tmin;       // θ bounds (nullptr: θ used as given)
    const float* tmax;
    const int32_t* feat;     // [16] state slot of conditioner feature k (n + d → zero)
    const int32_t* af;       // [n_af] state slots of the transformed dims
    float* zbar;             // [sample][d] adjoint of the layer output, updated in place
    float* ebuf;             // [sample][4] exp(-s) from the s-net launch
    float* partial;          // [workgroup][p_total] gradient partials
    const uint8_t* blob;     // chain weight blob (forward fragments)
    const uint8_t* tblob;    // transposed fragments
    const uint8_t* sblob;    // SPLIT: the chain's SPLIT blob (forward region of the net)
    const uint8_t* tsblob;   // SPLIT: the trainer's W1ᵀ planes
    int64_t batch;
    int64_t p_total;
    int d, n, n_af, kind, phase;
    float inv_n;             // 1 / (global batch size)
    GNet net;
};

size_t train_net_lds(int ht, const GNet& g);
hipError_t set_train_lds_limit(size_t lds);
hipError_t launch_train_net(int ht, int nh, int am, const TrainArgs& a, unsigned grid, size_t lds,
                            hipStream_t st);
hipError_t train_net_occupancy(int ht, int nh, int am, size_t lds, int* blocks, bool split = false);

hipError_t launch_scale(float* dst, const float* src, float s, int64_t count, hipStream_t st);
hipError_t launch_norm_adjoint(float* zbar, const float* xmin, const float* xmax, float alpha, float beta, int d,
                               int64_t batch, hipStream_t st);
hipError_t launch_reduce_grads(const float* partial, int n_parts, int64_t p_total, float* grad, hipStream_t st);
// Adam update with βᵗ read from bt[0..1] on the device, then βᵗ .*= β (one more launch).
hipError_t launch_adam(float* x, const float* g, float* m, float* v, int64_t count, float eta, float b1, float b2,
                       float eps, float* bt, hipStream_t st);
hipError_t launch_repack(float* blob, const int32_t* dst, const int32_t* src, int64_t count, const float* params,
                         hipStream_t st);
// SPLIT blob: byte offset dst[i] ← bf16 plane (src[i] & 3) of params[src[i] >> 2] (plane 3: the f32 value)
hipError_t launch_repack_split(uint8_t* blob, const int32_t* dst, const int32_t* src, int64_t count,
                               const float* params, hipStream_t st);

}  // namespace df
