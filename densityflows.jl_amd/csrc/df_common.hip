// df_common.hip — variant dispatch and the deterministic NLL partial reduction.
#include <hip/hip_runtime.h>

#include "df_kernels.h"

namespace df {

// Fixed-order sum of per-workgroup fp64 partials (bitwise reproducible).
__global__ void __launch_bounds__(256) reduce_partials_kernel(const double* part, int64_t n, double* out) {
    __shared__ double red[256];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

hipError_t launch_reduce_partials(const double* part, int64_t n, double* out, hipStream_t st) {
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(256), 0, st, part, n, out);
    return hipGetLastError();
}

hipError_t set_kernel_lds_limit(int ht, bool uniform, size_t lds) {
    if (uniform) {
        switch (ht) {
            case 1: return set_uniform_lds_limit_ht<1>(lds);
            case 2: return set_uniform_lds_limit_ht<2>(lds);
            case 4: return set_uniform_lds_limit_ht<4>(lds);
            default: return hipErrorInvalidValue;
        }
    }
    switch (ht) {
        case 1: return set_lds_limit_ht<1>(lds);
        case 2: return set_lds_limit_ht<2>(lds);
        case 4: return set_lds_limit_ht<4>(lds);
        case 8: return set_lds_limit_ht<8>(lds);
        case 16: return set_lds_limit_ht<16>(lds);
        default: return hipErrorInvalidValue;
    }
}

hipError_t kernel_occupancy(int ht, int mode, bool outv, int uniform, size_t lds, int* blocks) {
    if (uniform) {
        const int v = (outv ? 1 : 0) | (uniform >= 2 ? 2 : 0) | (uniform >= 3 ? 4 : 0) | (uniform == 4 ? 8 : 0);
        switch (ht) {
            case 1: return uniform_occupancy_ht<1>(mode, v, lds, blocks);
            case 2: return uniform_occupancy_ht<2>(mode, v, lds, blocks);
            case 4: return uniform_occupancy_ht<4>(mode, v, lds, blocks);
            default: return hipErrorInvalidValue;
        }
    }
    switch (ht) {
        case 1: return chain_occupancy_ht<1>(mode, outv, lds, blocks);
        case 2: return chain_occupancy_ht<2>(mode, outv, lds, blocks);
        case 4: return chain_occupancy_ht<4>(mode, outv, lds, blocks);
        case 8: return chain_occupancy_ht<8>(mode, outv, lds, blocks);
        case 16: return chain_occupancy_ht<16>(mode, outv, lds, blocks);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_chain(int ht, int mode, bool outv, int uniform, const ChainArgs& a, unsigned grid, size_t lds,
                        hipStream_t st) {
    if (uniform) {
        const int v = (outv ? 1 : 0) | (uniform >= 2 ? 2 : 0) | (uniform >= 3 ? 4 : 0) | (uniform == 4 ? 8 : 0);
        switch (ht) {
            case 1: return launch_uniform_ht<1>(mode, v, a, grid, lds, st);
            case 2: return launch_uniform_ht<2>(mode, v, a, grid, lds, st);
            case 4: return launch_uniform_ht<4>(mode, v, a, grid, lds, st);
            default: return hipErrorInvalidValue;
        }
    }
    switch (ht) {
        case 1: return launch_chain_ht<1>(mode, outv, a, grid, lds, st);
        case 2: return launch_chain_ht<2>(mode, outv, a, grid, lds, st);
        case 4: return launch_chain_ht<4>(mode, outv, a, grid, lds, st);
        case 8: return launch_chain_ht<8>(mode, outv, a, grid, lds, st);
        case 16: return launch_chain_ht<16>(mode, outv, a, grid, lds, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace df
