// df_sample.hip — sample(flow, dims, θ) on the device (src/Flows.jl:157-192):
// the base draw r ~ MvNormal(0, I) (Flows.jl:114) from a counter-based Philox4x32-10
// stream, then the fused forward! (df_flow_forward_inplace) with θ normalised in the
// kernel.  The NTuple θ method (Flows.jl:178-188, collect(θ) .* ones(T, (1, dims...)))
// broadcasts one n-vector into a per-chain workspace first.
//
// Stream: element k of the (d, batch) draw comes from Philox4x32-10 with key = seed and
// counter = (offset + k/4, 0, 0, 0), output word k%4; words (0,1) and (2,3) are Box-Muller
// pairs: u = (w >> 8) · 2^-24 + 2^-25 ∈ (0, 1), z = sqrt(-2 ln u_a)·(cos, sin)(2π u_b).
// Julia's Xoshiro stream cannot be matched; parity is tested on the draw
// read back through df_random_normal.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "densityflows_hip.h"
#include "df_handle.h"

namespace df {
namespace {

struct U4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

__device__ __forceinline__ float unit_open(uint32_t w) {  // (0, 1), never 0 or 1
    return (float)(w >> 8) * 5.9604644775390625e-08f + 2.98023223876953125e-08f;
}

__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
    const float r = sqrtf(-2.f * logf(unit_open(a)));
    float s, c;
    sincosf(6.28318530717958647692f * unit_open(b), &s, &c);
    z0 = r * c;
    z1 = r * s;
}

// One thread: the 4 elements of counter i (vector store when the 4 lie inside `count`).
__global__ void __launch_bounds__(256) normal_kernel(float* out, int64_t count, uint32_t k0, uint32_t k1,
                                                      uint64_t offset) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t k = 4 * i;
    if (k >= count) return;
    const uint64_t ctr = offset + (uint64_t)i;
    const U4 w = philox4x32_10(U4{(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u}, k0, k1);
    float z[4];
    box_muller(w.x, w.y, z[0], z[1]);
    box_muller(w.z, w.w, z[2], z[3]);
    if (k + 4 <= count && (reinterpret_cast<uintptr_t>(out + k) & 15) == 0) {
        *reinterpret_cast<float4*>(out + k) = float4{z[0], z[1], z[2], z[3]};
    } else {
        for (int e = 0; e < 4 && k + e < count; ++e) out[k + e] = z[e];
    }
}

__global__ void __launch_bounds__(256) broadcast_kernel(float* dst, const float* v, int n, int64_t batch) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < (int64_t)n * batch) dst[i] = v[i % n];
}

hipError_t launch_normal(float* out, int64_t count, uint64_t seed, uint64_t offset, hipStream_t st) {
    const int64_t threads = (count + 3) / 4;
    if (threads == 0) return hipSuccess;
    const int64_t blocks = (threads + 255) / 256;
    if (blocks > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(normal_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, count, (uint32_t)seed,
                       (uint32_t)(seed >> 32), offset);
    return hipGetLastError();
}

}  // namespace
}  // namespace df

using namespace df::api;

extern "C" {

int df_random_normal(float* out, int64_t count, uint64_t seed, uint64_t offset, void* stream) {
    if (count < 0) return set_err(DF_ERR_SHAPE, "negative count");
    if (count > 0 && !out) return set_err(DF_ERR_INVALID, "null output");
    hipError_t e = df::launch_normal(out, count, seed, offset, (hipStream_t)stream);
    return e == hipSuccess ? DF_OK : hip_err(e, "normal_kernel launch");
}

int df_flow_sample(df_chain* c, float* x_out, const float* theta_raw, int theta_broadcast, int64_t batch,
                   uint64_t seed, uint64_t offset, void* stream) {
    if (!c) return set_err(DF_ERR_INVALID, "null chain");
    if (batch < 0) return set_err(DF_ERR_SHAPE, "negative batch size");
    if (batch == 0) return DF_OK;
    if (!x_out) return set_err(DF_ERR_INVALID, "null output array");
    const int d = c->plan.d, n = c->plan.n;
    if (n > 0 && !theta_raw)
        return set_err(DF_ERR_SHAPE, "dimensions θ must match (n, dims...) with n number of trained parameters");
    if (n > 0 && !c->has_bounds) return set_err(DF_ERR_INVALID, "θ bounds not set (df_chain_set_theta_bounds)");
    DeviceGuard gd(c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = df::launch_normal(x_out, (int64_t)d * batch, seed, offset, st);
    if (e != hipSuccess) return hip_err(e, "normal_kernel launch");
    const float* th = theta_raw;
    if (n > 0 && theta_broadcast) {
        const int64_t need = (int64_t)n * batch;
        if (need > c->theta_ws_cap) {
            if (c->d_theta_ws) {
                // the workspace belongs to the chain, not to a stream: an earlier sample on
                // any stream may still read it
                e = hipDeviceSynchronize();
                if (e != hipSuccess) return hip_err(e, "hipDeviceSynchronize");
                (void)hipFree(c->d_theta_ws);
            }
            c->d_theta_ws = nullptr;
            c->theta_ws_cap = 0;
            e = hipMalloc(reinterpret_cast<void**>(&c->d_theta_ws), sizeof(float) * need);
            if (e != hipSuccess) return set_err(DF_ERR_NOMEM, "hipMalloc failed (θ broadcast)");
            c->theta_ws_cap = need;
        }
        hipLaunchKernelGGL(df::broadcast_kernel, dim3((unsigned)((need + 255) / 256)), dim3(256), 0, st,
                           c->d_theta_ws, theta_raw, n, batch);
        if ((e = hipGetLastError()) != hipSuccess) return hip_err(e, "broadcast_kernel launch");
        th = c->d_theta_ws;
    }
    return df_flow_forward_inplace(c, x_out, th, batch, stream);
}

}  // extern "C"
