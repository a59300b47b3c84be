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

// 16-sample MFMA column tiles per wave for a kernel variant (must match the
// planner: Plan::tiles).
#ifndef DF_TILES_SMALL
#define DF_TILES_SMALL 1
#endif
constexpr int tiles_per_wave(int ht) { return ht <= 4 ? DF_TILES_SMALL : 1; }

struct ChainArgs {
    const float* zin;
    const float* theta;
    float* xout;
    float* ldj_out;
    float* lp_out;
    double* partial;
    int64_t batch;
    const DevLayer* layers;
    const DevDense* denses;
    const DevChunk* chunks;
    const DevStage* stages;
    const uint8_t* blob;
    const int32_t* tables;
    const float* params;
    const float* tmin;   // θ bounds; nullptr → θ used as given
    const float* tmax;
    int d, n, stride, n_layers;
    int tab_ints;
    int tab_bytes;       // LDS bytes reserved for tables (16-B multiple)
    int stage_bytes;     // LDS bytes reserved for the stage buffer (16-B multiple)
    float c0;            // -(d·log2π)/2
};

// Per-variant entry points (explicitly instantiated in df_kernels_ht*.hip).
template <int HT>
hipError_t launch_chain_ht(int mode, bool outv, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st);
template <int HT>
hipError_t set_lds_limit_ht(size_t lds);

// Dispatch over the variant (df_common.hip).
hipError_t set_kernel_lds_limit(int ht, size_t lds);
hipError_t launch_chain(int ht, int mode, bool outv, const ChainArgs& a, unsigned grid, size_t lds,
                        hipStream_t st);
hipError_t launch_reduce_partials(const double* part, int64_t n, double* out, hipStream_t st);

}  // namespace df
