// df_train.hip — training kernels: the per-net reverse sweep (df_train_impl.h,
// instantiated for hidden widths 16/32/64 and 0 or 1 hidden Dense), and the
// element-wise steps around it (z̄ seed, NormalizationLayer adjoint, the
// fixed-order gradient reduction, Adam, weight regathering).
#include "df_train_impl.h"

namespace df {

namespace {

#ifndef DF_TRAIN_NAF
#define DF_TRAIN_NAF 1
#endif
// naf: the transformed-dim count; the SPLIT instances for 2 and 3 (d = 5 chains) have it
// at compile time (DF_TRAIN_NAF)
void* train_ptr(int ht, int nh, int am, bool split = false, int naf = 0) {
    if (split) {
        if (nh != 1 || am != trn::AM_RELU) return nullptr;
        const int nf = DF_TRAIN_NAF ? naf : 0;
        if (ht == 2) return nf == 2 ? train_kernel_ptr<2, 1, trn::AM_RELU, true, 2>()
                            : nf == 3 ? train_kernel_ptr<2, 1, trn::AM_RELU, true, 3>()
                                      : train_kernel_ptr<2, 1, trn::AM_RELU, true>();
        if (ht == 4) return nf == 2 ? train_kernel_ptr<4, 1, trn::AM_RELU, true, 2>()
                            : nf == 3 ? train_kernel_ptr<4, 1, trn::AM_RELU, true, 3>()
                                      : train_kernel_ptr<4, 1, trn::AM_RELU, true>();
        return nullptr;
    }
#define DF_T(H)                                                                                           \
    (nh ? (am == trn::AM_RELU ? train_kernel_ptr<H, 1, trn::AM_RELU>()                                   \
                              : (am == trn::AM_PRE ? train_kernel_ptr<H, 1, trn::AM_PRE>()                \
                                                   : train_kernel_ptr<H, 1, trn::AM_Y>()))                \
        : (am == trn::AM_RELU ? train_kernel_ptr<H, 0, trn::AM_RELU>()                                   \
                              : (am == trn::AM_PRE ? train_kernel_ptr<H, 0, trn::AM_PRE>()                \
                                                   : train_kernel_ptr<H, 0, trn::AM_Y>())))
    switch (ht) {
        case 1: return DF_T(1);
        case 2: return DF_T(2);
        case 4: return DF_T(4);
        default: return nullptr;
    }
#undef DF_T
}

// z̄ = z / N
__global__ void scale_kernel(float* dst, const float* src, float s, int64_t count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[i] = src[i] * s;
}

// NormalizationLayer inverse z = (β(x - x_min) + α(x_max - x)) / x_diff
// (src/norm/Normalization.jl:66-76):  x̄ = z̄ · (β - α) / x_diff
__global__ void norm_adjoint_kernel(float* zbar, const float* xmin, const float* xmax, float alpha, float beta,
                                    int d, int64_t count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) {
        const int c = (int)(i % d);
        zbar[i] = zbar[i] * ((beta - alpha) / (xmax[c] - xmin[c]));
    }
}

// ∇[p] = Σ_w partial[w][p], w in increasing order (bitwise reproducible)
__global__ void reduce_grads_kernel(const float* partial, int n_parts, int64_t p_total, float* grad) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= p_total) return;
    float s = 0.f;
    for (int w = 0; w < n_parts; ++w) s += partial[(int64_t)w * p_total + p];
    grad[p] = s;
}

// The same sums, four parameters per thread (p_total % 4 == 0): 16-byte loads, eight
// partial rows in flight per thread; each sum still runs over w in increasing order.
__global__ void reduce_grads4_kernel(const float* partial, int n_parts, int64_t p_total, float* grad) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (p >= p_total) return;
    v4 s = v4{0.f, 0.f, 0.f, 0.f};
    int w = 0;
    for (; w + 8 <= n_parts; w += 8) {
        v4 r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = *reinterpret_cast<const v4*>(partial + (int64_t)(w + k) * p_total + p);
#pragma unroll
        for (int k = 0; k < 8; ++k) s = s + r[k];
    }
    for (; w < n_parts; ++w) s = s + *reinterpret_cast<const v4*>(partial + (int64_t)w * p_total + p);
    *reinterpret_cast<v4*>(grad + p) = s;
}

// Optimisers.Adam (apply!, Optimisers.jl v0.4):
//   m = β1 m + (1-β1) g;  v = β2 v + (1-β2) g²
//   x -= m / (1-β1ᵗ) / (sqrt(v / (1-β2ᵗ)) + ϵ) · η          (all Float32)
// βᵗ lives on the device (bt[0], bt[1]) so that a captured train step (hipGraph)
// replays with the current power; adam_advance_kernel moves it on after the update.
__global__ void adam_kernel(float* x, const float* g, float* m, float* v, int64_t count, float eta, float b1,
                            float b2, float eps, const float* bt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float bt1 = bt[0], bt2 = bt[1];
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * (gi * gi);
    m[i] = mi;
    v[i] = vi;
    const float upd = mi / (1.f - bt1) / (sqrtf(vi / (1.f - bt2)) + eps) * eta;
    x[i] = x[i] - upd;
}

__global__ void adam_advance_kernel(float* bt, float b1, float b2) {
    if (threadIdx.x == 0) {
        bt[0] = bt[0] * b1;  // βᵗ .* β in Float32 (Optimisers.Adam)
        bt[1] = bt[1] * b2;
    }
}

__global__ void repack_kernel(float* blob, const int32_t* dst, const int32_t* src, int64_t count,
                              const float* params) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) blob[dst[i]] = params[src[i]];
}

__global__ void repack_split_kernel(uint8_t* blob, const int32_t* dst, const int32_t* src, int64_t count,
                                    const float* params) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int32_t code = src[i];
    const float v = params[code >> 2];
    const int plane = code & 3;
    if (plane == 3) *reinterpret_cast<float*>(blob + dst[i]) = v;
    else *reinterpret_cast<uint16_t*>(blob + dst[i]) = bf16_split_plane(v, plane);
}

unsigned blocks_for(int64_t count, int threads) { return (unsigned)((count + threads - 1) / threads); }

}  // namespace

size_t train_net_lds(int ht, const GNet& g) {
    const size_t tarea = (size_t)kTrainWaves * 2 * 16 * ht * kTS * 4;
    // the reduction: the net's trainables + dW0 / dW1 / dW_out in padded regions
    // (train_net_kernel; generous bounds: n_in, n_out <= 16, dW1 rows <= h + 8 apart)
    const size_t h = (size_t)g.h_true;
    const size_t red = (((size_t)g.p_count + 3) + (h + 1) * 16 + 3 + h * (h + 8) + 3 + 17 * h) * 4;
    if (g.split) return (size_t)g.sfwd_bytes + ht * 1024 + g.st_bytes + (tarea > red ? tarea : red);
    return (size_t)g.fwd_bytes + g.t_bytes + (tarea > red ? tarea : red);
}

hipError_t set_train_lds_limit(size_t lds) {
    for (int ht : {1, 2, 4})
        for (int nh = 0; nh < 2; ++nh)
            for (int am = 0; am < 3; ++am) {
                hipError_t e = hipFuncSetAttribute(train_ptr(ht, nh, am),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                if (e != hipSuccess) return e;
            }
    for (int ht : {2, 4}) {
        for (int naf : {0, 2, 3}) {
            hipError_t e = hipFuncSetAttribute(train_ptr(ht, 1, trn::AM_RELU, true, naf),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

hipError_t launch_train_net(int ht, int nh, int am, const TrainArgs& a, unsigned grid, size_t lds,
                            hipStream_t st) {
    // out_valu<NO = NAF> needs n_out = n_af, the 4x4x1 x̄ at most 4 conditioner inputs
    const int naf = (a.net.split && a.net.su.n_out == a.n_af && a.net.n_in <= 4) ? a.n_af : 0;
    void* k = train_ptr(ht, nh, am, a.net.split != 0, naf);
    if (!k) return hipErrorInvalidValue;
    void* args[] = {const_cast<TrainArgs*>(&a)};
    return hipLaunchKernel(k, dim3(grid), dim3(train_threads(a.net.split != 0)), args, lds, st);
}

hipError_t train_net_occupancy(int ht, int nh, int am, size_t lds, int* blocks, bool split) {
    void* k = train_ptr(ht, nh, am, split);
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, k, train_threads(split), lds);
}

hipError_t launch_scale(float* dst, const float* src, float s, int64_t count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, st, dst, src, s, count);
    return hipGetLastError();
}

hipError_t launch_norm_adjoint(float* zbar, const float* xmin, const float* xmax, float alpha, float beta, int d,
                               int64_t batch, hipStream_t st) {
    const int64_t count = batch * d;
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(norm_adjoint_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, st, zbar, xmin, xmax,
                       alpha, beta, d, count);
    return hipGetLastError();
}

hipError_t launch_reduce_grads(const float* partial, int n_parts, int64_t p_total, float* grad, hipStream_t st) {
    if (p_total <= 0) return hipSuccess;
    if (p_total % 4 == 0 && (reinterpret_cast<uintptr_t>(partial) % 16) == 0 && (reinterpret_cast<uintptr_t>(grad) % 16) == 0)
        hipLaunchKernelGGL(reduce_grads4_kernel, dim3(blocks_for(p_total / 4, 256)), dim3(256), 0, st, partial,
                           n_parts, p_total, grad);
    else
        hipLaunchKernelGGL(reduce_grads_kernel, dim3(blocks_for(p_total, 256)), dim3(256), 0, st, partial, n_parts,
                           p_total, grad);
    return hipGetLastError();
}

hipError_t launch_adam(float* x, const float* g, float* m, float* v, int64_t count, float eta, float b1, float b2,
                       float eps, float* bt, hipStream_t st) {
    if (count > 0)
        hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, st, x, g, m, v, count, eta, b1, b2,
                           eps, static_cast<const float*>(bt));
    hipLaunchKernelGGL(adam_advance_kernel, dim3(1), dim3(64), 0, st, bt, b1, b2);
    return hipGetLastError();
}

hipError_t launch_repack(float* blob, const int32_t* dst, const int32_t* src, int64_t count, const float* params,
                         hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(repack_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, st, blob, dst, src, count, params);
    return hipGetLastError();
}

hipError_t launch_repack_split(uint8_t* blob, const int32_t* dst, const int32_t* src, int64_t count,
                               const float* params, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(repack_split_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, st, blob, dst, src, count,
                       params);
    return hipGetLastError();
}

}  // namespace df
