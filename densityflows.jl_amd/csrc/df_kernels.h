// df_kernels.h — launch interface of the fused chain kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "df_plan.h"

namespace df {

enum : int {
    MODE_FWD = 0,          // forward(chain, z, θ) -> (x, ldj)
    MODE_FWD_INPLACE = 1,  // forward!(chain, z, θ)
    MODE_BWD = 2,          // backward(chain, x, θ) -> (z, ldj)
    MODE_LOGPDF = 3        // backward + MvNormal(0, I) logpdf + ldj
};

struct ChainArgs {
    const float* zin;
    const float* theta;
    float* xout;
    float* ldj_out;
    float* lp_out;
    double* partial;
    int64_t batch;
    const DevLayer* layers;
    const ULayer* ulayers;   // specialised kernel only
    const DevDense* denses;
    const DevChunk* chunks;
    const DevStage* stages;
    const uint8_t* blob;
    const int32_t* tables;
    const float* params;
    const float* tmin;   // θ bounds; nullptr → θ used as given
    const float* tmax;
    int d, n, stride, n_layers;
    int tiles;           // 16-sample tiles per wave resident in LDS (Plan::tiles)
    int tab_ints;
    int tab_bytes;       // LDS bytes reserved for tables (16-B multiple; specialised kernel: + n_par bounds)
    int n_par;           // specialised kernel: floats of `params` copied to LDS after the tables
    int stage_bytes;     // LDS bytes of ONE stage buffer (multiple of 1 KiB)
    int n_stage_bufs;    // 1 (single-stage chain) or 2 (double-buffered)
    const int32_t* sched_fwd;
    const int32_t* sched_bwd;
    int n_sched_fwd;
    int n_sched_bwd;
    float c0;            // -(d·log2π)/2
    float* snap;         // inverse modes: state after each layer, [layer][sample][d]
    float* hsave;        // inverse modes, generic kernel: hidden activations of every net,
                         // [(layer·2 + net)·hsave_h + k][sample][hsave_w] (training, layer-wise path)
    int hsave_w, hsave_h;
    float* fsave;        // inverse modes, wide SPLIT kernel (training, H0 recomputed): the first
                         // Dense's input vcat(θ, u)[axis_nn] of every net, [layer·2 + net][sample][32],
                         // and hsave then keeps H1 only (hsave_h = 1)
    const WLayer* wlayers;   // wide-net kernel only (stages / blob / schedules then refer to the wide blob)
    const float* wbias;
    uint64_t* clk;           // effective-clock stamps (df_chain_clock_probe), nullptr = off
};

// Effective shader clock of a launch (df_chain_clock_probe): wave 0 of every
// workgroup adds Δs_memtime (shader cycles) and Δs_memrealtime (100 MHz ticks)
// over its lifetime to clk[2·blockIdx.x + {0, 1}].  Launches on one stream do
// not overlap, so the read-modify-write needs no atomics; the values go to a
// buffer nothing else reads.  Off (clk == nullptr): one scalar branch per end.
struct ClockStamp {
    uint64_t t0 = 0, r0 = 0;
    __device__ __forceinline__ void begin(const ChainArgs& a) {
        if (a.clk) {
            t0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
        }
    }
    __device__ __forceinline__ void end(const ChainArgs& a) {
        if (a.clk && threadIdx.x == 0) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
            uint64_t* p = a.clk + 2 * (uint64_t)blockIdx.x;
            p[0] += t1 - t0;
            p[1] += r1 - r0;
        }
    }
};

// Per-variant entry points (explicitly instantiated in df_kernels_ht*.hip).
template <int HT>
hipError_t launch_chain_ht(int mode, bool outv, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st);
template <int HT>
hipError_t set_lds_limit_ht(size_t lds);
template <int HT>
hipError_t launch_uniform_ht(int mode, int variant, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st);
template <int HT>
hipError_t set_uniform_lds_limit_ht(size_t lds);
template <int HT>
hipError_t uniform_occupancy_ht(int mode, int variant, size_t lds, int* blocks);
template <int HT>
hipError_t chain_occupancy_ht(int mode, bool outv, size_t lds, int* blocks);

// Dispatch over the variant (df_common.hip).
hipError_t set_kernel_lds_limit(int ht, bool uniform, size_t lds);
// uniform: 0 = generic kernel, 1 = specialised, 2 = specialised relu-only, 3 = FAST,
// 4 = FAST on the bf16x3 split stages (SPLIT)
hipError_t launch_chain(int ht, int mode, bool outv, int uniform, const ChainArgs& a, unsigned grid,
                        size_t lds, hipStream_t st);
hipError_t kernel_occupancy(int ht, int mode, bool outv, int uniform, size_t lds, int* blocks);
hipError_t launch_reduce_partials(const double* part, int64_t n, double* out, hipStream_t st);

// Wide-net kernel (df_wide.hip): 4-wave workgroups of kWideWaves*16*kWideT samples.
// split: the SPLIT variant (bf16x3 products; a.blob / stages / schedules / wlayers / tables are the split ones)
hipError_t launch_wide(int mode, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st, bool split = false);
hipError_t set_wide_lds_limit(size_t lds, bool split = false);

// Small-batch kernel (df_small.hip): FAST exact-f32 chains of hidden 16 with n + d <= 8 and
// at most kSmallLayers layers; one wave of 16 samples per workgroup.
constexpr int kSmallSamples = 16;
constexpr int kSmallLayers = 4;
// Everything the small-batch kernel reads besides the blob and the batch arrays, passed
// BY VALUE as a kernel argument: it arrives with the kernel arguments, so the weight
// loads need no dependent scalar-memory round trips (descriptor → stage → fragments)
// before they can issue.  Built on the host from the plan (df_capi.hip small_desc).
struct SmallDesc {
    int32_t w0[kSmallLayers][2], wh[kSmallLayers][2], wo[kSmallLayers][2];  // blob byte offsets, net s / t
    int8_t kind[kSmallLayers], elem_start[kSmallLayers], elem_end[kSmallLayers], n_out[kSmallLayers];
    int8_t feat[kSmallLayers][4];  // state columns of the conditioner features k = lane group
    int8_t af[kSmallLayers][4];    // state columns of the transformed dims
    float alpha[kSmallLayers], beta[kSmallLayers], ldj_const[kSmallLayers];
    float xmin[kSmallLayers][8], xmax[kSmallLayers][8];  // NormalizationLayer bounds (d <= 8)
    // (the θ bounds are NOT here: the kernel reads them through ChainArgs::tmin / tmax, the
    // chain's device copy, so a captured train step sees df_chain_set_theta_bounds)
};
// nw = 2 (default): the s- and t-nets of a layer on two waves of the workgroup; 1: one wave
hipError_t launch_small(int mode, const ChainArgs& a, const SmallDesc& sd, unsigned grid, hipStream_t st,
                        int nw = 2);

}  // namespace df
