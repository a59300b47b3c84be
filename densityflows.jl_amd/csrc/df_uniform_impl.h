// df_uniform_impl.h — the specialised fused kernel for chains whose coupling
// layers all use the reference's default conditioner shape (_dflt_net,
// src/Layers.jl:33-50): Dense(in, H, σ), nh × Dense(H, H, σ), Dense(H, out),
// with H = 16·HT exactly, in <= 16, and each net resident in ONE LDS stage.
// Same numerics and data flow as the generic kernel (df_chain_impl.h) with
// every width known at compile time: no per-tile guards, ping-pong
// accumulators instead of register copies, compact per-net descriptors.
#pragma once

#include "df_chain_impl.h"

namespace df {
namespace uni {


using impl::lds4;
using impl::mfma4;
using impl::Stager;

__device__ __forceinline__ float relu_fast(float x) { return __builtin_fmaxf(x, 0.f); }

// acc = W·x (+ b), x = the state features vcat(θ,z)[axis_nn] (<= 16 of them).
template <int HT>
__device__ __forceinline__ void dense_first(const uint8_t* buf, const UNet& N, const float (&xin)[4],
                                            f32x4 (&acc)[HT]) {
    const int lane = threadIdx.x & 63;
    const uint8_t* wb = buf + N.off_w0 + lane * 16;
#pragma unroll
    for (int m = 0; m < HT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 w[HT];
#pragma unroll
    for (int m = 0; m < HT; ++m) w[m] = lds4(wb + m * 1024);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (r < N.ks) {
#pragma unroll
            for (int m = 0; m < HT; ++m) acc[m] = mfma4(w[m][r], xin[r], acc[m]);
        }
    }
}

// out = W·in over a full H×H Dense (fragments [kq][m][lane][4] at wb).
template <int HT>
__device__ __forceinline__ void dense_hidden(const uint8_t* wb, const f32x4 (&in)[HT], f32x4 (&out)[HT]) {
    const int lane = threadIdx.x & 63;
    wb += lane * 16;
    constexpr int MB = HT < 4 ? HT : 4;
#pragma unroll
    for (int m = 0; m < HT; ++m) out[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m0 = 0; m0 < HT; m0 += MB) {
        f32x4 w[2][MB];
#pragma unroll
        for (int mm = 0; mm < MB; ++mm) w[0][mm] = lds4(wb + (m0 + mm) * 1024);
#pragma unroll
        for (int kq = 0; kq < HT; ++kq) {
            const int cb = kq & 1;
            if (kq + 1 < HT) {
#pragma unroll
                for (int mm = 0; mm < MB; ++mm) w[cb ^ 1][mm] = lds4(wb + ((kq + 1) * HT + m0 + mm) * 1024);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int mm = 0; mm < MB; ++mm) out[m0 + mm] = mfma4(w[cb][mm][r], in[kq][r], out[m0 + mm]);
        }
    }
}

// v = σ.(v .+ b)  — bias after the product (Flux: W*x .+ b)
template <int HT>
__device__ __forceinline__ void bias_act(const uint8_t* bb, int act, f32x4 (&v)[HT]) {
    const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int m = 0; m < HT; ++m) v[m] = v[m] + lds4(bb + ((16 * m + 4 * g) << 2));
    if (act == DF_ACT_RELU) {
#pragma unroll
        for (int m = 0; m < HT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[m][r] = relu_fast(v[m][r]);
    } else if (act != DF_ACT_IDENTITY) {
#pragma unroll
        for (int m = 0; m < HT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[m][r] = impl::act_fn(act, v[m][r]);
    }
}

// Final Dense, <= 4 outputs, as a VALU GEMV; every lane ends with all outputs.
template <int HT>
__device__ __forceinline__ f32x4 out_valu(const uint8_t* buf, const UNet& N, const f32x4 (&h)[HT]) {
    const int g = (threadIdx.x & 63) >> 4;
    const uint8_t* w3 = buf + N.off_out;
    constexpr int INP = 16 * HT;
    const float* b3 = reinterpret_cast<const float*>(w3) + N.n_out * INP;
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oo = 0; oo < 4; ++oo) {
        if (oo < N.n_out) {
            float p = 0.f;
#pragma unroll
            for (int kq = 0; kq < HT; ++kq) {
                const f32x4 w = lds4(w3 + ((oo * INP + 16 * kq + 4 * g) << 2));
#pragma unroll
                for (int r = 0; r < 4; ++r) p = __builtin_fmaf(w[r], h[kq][r], p);
            }
            p += __shfl_xor(p, 16);
            p += __shfl_xor(p, 32);
            float v = p + b3[oo];
            o[oo] = (N.act_out == DF_ACT_IDENTITY) ? v : impl::act_fn(N.act_out, v);
        }
    }
    return o;
}

// Final Dense through MFMA (out <= 32): rows 16m + 4g + r in out[m].
template <int HT>
__device__ __forceinline__ void out_mfma(const uint8_t* buf, const UNet& N, const f32x4 (&h)[HT],
                                         f32x4 (&out)[2]) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const uint8_t* wb = buf + N.off_out + lane * 16;
    const int mt = (N.n_out + 15) >> 4;
    out[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    out[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kq = 0; kq < HT; ++kq) {
        const f32x4 w0 = lds4(wb + (kq * mt + 0) * 1024);
#pragma unroll
        for (int r = 0; r < 4; ++r) out[0] = mfma4(w0[r], h[kq][r], out[0]);
        if (mt > 1) {
            const f32x4 w1 = lds4(wb + (kq * mt + 1) * 1024);
#pragma unroll
            for (int r = 0; r < 4; ++r) out[1] = mfma4(w1[r], h[kq][r], out[1]);
        }
    }
    const uint8_t* bb = buf + N.off_out + HT * mt * 1024;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        if (m < mt) {
            f32x4 v = out[m] + lds4(bb + ((16 * m + 4 * g) << 2));
            if (N.act_out != DF_ACT_IDENTITY)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = impl::act_fn(N.act_out, v[r]);
            out[m] = v;
        }
    }
}

// Evaluate net N for one 16-sample tile (state rows at `ro`) and apply its
// coupling phase; returns Σ_k s_k for s phases (row order), 0 otherwise.
template <int HT, bool OUTV, int PH>
__device__ __forceinline__ float net_tile(const uint8_t* buf, const UNet& N, const ULayer& L, const int32_t* tab,
                                          float* state, int ro) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    constexpr bool SPH = (PH == impl::PH_S_FWD || PH == impl::PH_S_BWD);
    // conditioner input: features k = 4r + g of vcat(θ,z)[axis_nn] (zero slot pads)
    float xin[4];
    const int32_t* feat = tab + L.feat_tab;
#pragma unroll
    for (int r = 0; r < 4; ++r) xin[r] = (r < N.ks) ? state[ro + feat[4 * r + g]] : 0.f;

    f32x4 A[HT], B[HT];
    dense_first<HT>(buf, N, xin, A);
    bias_act<HT>(buf + N.off_b0, N.act0, A);
    // hidden Denses alternate A -> B -> A ... (no register copies)
    bool in_a = true;
    for (int k = 0; k < N.nh; k += 2) {
        dense_hidden<HT>(buf + N.off_h + k * N.hstride, A, B);
        bias_act<HT>(buf + N.off_h + k * N.hstride + HT * HT * 1024, N.acth, B);
        in_a = false;
        if (k + 1 < N.nh) {
            dense_hidden<HT>(buf + N.off_h + (k + 1) * N.hstride, B, A);
            bias_act<HT>(buf + N.off_h + (k + 1) * N.hstride + HT * HT * 1024, N.acth, A);
            in_a = true;
        }
    }
    const int32_t* af = tab + L.af_tab;
    float sum = 0.f;
    if constexpr (OUTV) {
        const f32x4 o = in_a ? out_valu<HT>(buf, N, A) : out_valu<HT>(buf, N, B);
        const float y = impl::sel4(o, g);
        if (g < L.n_af) {
            const int slot = af[g];
            float v = state[ro + slot];
            if (PH == impl::PH_S_FWD) v = v * expf(y);
            if (PH == impl::PH_T_FWD) v = v + y;
            if (PH == impl::PH_T_BWD) v = v - y;
            if (PH == impl::PH_S_BWD) v = v * expf(-y);
            state[ro + slot] = v;
        }
        if (SPH) {
            // ldj = Σ_k s[k] in row order (RNVP.jl:180 / :86)
            sum = o[0];
#pragma unroll
            for (int oo = 1; oo < 4; ++oo)
                if (oo < L.n_af) sum = sum + o[oo];
        }
    } else {
        f32x4 o[2];
        if (in_a) out_mfma<HT>(buf, N, A, o);
        else out_mfma<HT>(buf, N, B, o);
        float p = 0.f;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int oo = 16 * m + 4 * g + r;
                if (oo < L.n_af) {
                    const int slot = af[oo];
                    const float y = o[m][r];
                    float v = state[ro + slot];
                    if (PH == impl::PH_S_FWD) v = v * expf(y);
                    if (PH == impl::PH_T_FWD) v = v + y;
                    if (PH == impl::PH_T_BWD) v = v - y;
                    if (PH == impl::PH_S_BWD) v = v * expf(-y);
                    state[ro + slot] = v;
                    if (SPH) p = p + y;
                }
            }
        if (SPH) {
            p += __shfl_xor(p, 16);
            p += __shfl_xor(p, 32);
            sum = p;
        }
    }
    return sum;
}

}  // namespace uni

template <int HT, int MODE, bool OUTV>
__global__ void __launch_bounds__(kBlockThreads, DF_WAVES_PER_EU(HT))
uniform_kernel(ChainArgs a) {
    using namespace uni;
    constexpr bool FWD = (MODE == MODE_FWD || MODE == MODE_FWD_INPLACE);
    constexpr bool WANT_LDJ = (MODE != MODE_FWD_INPLACE);

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int stage_area = a.stage_bytes * a.n_stage_bufs;
    int32_t* tab = reinterpret_cast<int32_t*>(smem + stage_area);
    float* state = reinterpret_cast<float*>(smem + stage_area + a.tab_bytes);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int d = a.d, n = a.n, stride = a.stride, nd = n + d;
    const int nt = a.tiles;
    const int S = kWavesPerBlock * 16 * nt;
    const int cA = nd + 1, cE = nd + 2;
    const int64_t s0 = (int64_t)blockIdx.x * S;
    const int nvalid = (int)((a.batch - s0) < S ? (a.batch - s0) : S);

    Stager sg;
    sg.base = smem;
    sg.bytes = a.stage_bytes;
    sg.sched = FWD ? a.sched_fwd : a.sched_bwd;
    sg.n = FWD ? a.n_sched_fwd : a.n_sched_bwd;
    impl::stager_start(sg, a);

    for (int i = tid; i < a.tab_ints; i += kBlockThreads) tab[i] = a.tables[i];
    for (int i = tid; i < S * d; i += kBlockThreads) {
        const int smp = i / d, c = i - smp * d;
        float v = 0.f;
        if (smp < nvalid) v = a.zin[(s0 + smp) * d + c];
        state[smp * stride + n + c] = v;
    }
    for (int i = tid; i < S * n; i += kBlockThreads) {
        const int smp = i / n, c = i - smp * n;
        float v = 0.f;
        if (smp < nvalid) {
            v = a.theta[(s0 + smp) * n + c];
            if (a.tmin) {  // normalize_input (Data.jl:213-218)
                const float lo = a.tmin[c], diff = a.tmax[c] - lo;
                v = (diff == 0.f) ? 0.f : (v - lo) / diff;
            }
        }
        state[smp * stride + c] = v;
    }
    for (int i = tid; i < S; i += kBlockThreads)
        for (int c = nd; c < stride; ++c) state[i * stride + c] = 0.f;
    __syncthreads();

    const int row0 = ((wave * nt) * 16 + j) * stride;  // tile tt: row0 + tt*16*stride
    const int tstep = 16 * stride;
    bool have_acc = false;

    auto ldj_update = [&](int ro, float l, bool first_in_elem, bool last_in_elem) {
        if (!WANT_LDJ || g != 0) return;
        const float e = first_in_elem ? l : state[ro + cE] + l;
        state[ro + cE] = e;
        if (last_in_elem) state[ro + cA] = have_acc ? state[ro + cA] + e : e;
    };

    for (int it = 0; it < a.n_layers; ++it) {
        const int li = FWD ? it : a.n_layers - 1 - it;
        const ULayer& L = a.ulayers[li];
        const int kind = L.kind;
        const bool first_in_elem = FWD ? L.elem_start : L.elem_end;
        const bool last_in_elem = FWD ? L.elem_end : L.elem_start;
        if (kind == DF_LAYER_NORM) {
            const float al = L.alpha, be = L.beta, delta = be - al;
            const float* xmn = a.params + L.norm_off;
            const float* xmx = xmn + d;
            for (int tt = 0; tt < nt; ++tt) {
                const int ro = row0 + tt * tstep;
                for (int i = g; i < d; i += 4) {
                    const float lo = xmn[i], hi = xmx[i], xd = hi - lo;
                    float v = state[ro + n + i];
                    if (FWD) v = ((xd * v - al * hi) + be * lo) / delta;
                    else v = (be * (v - lo) + al * (hi - v)) / xd;
                    state[ro + n + i] = v;
                }
                ldj_update(ro, FWD ? L.ldj_const : -L.ldj_const, first_in_elem, last_in_elem);
            }
        } else {
            const bool rnvp = (kind == DF_LAYER_RNVP);
            if (FWD) {
                if (rnvp) {
                    impl::ensure_stage(L.s.stage, sg, a);
                    const uint8_t* buf = sg.buf();
                    for (int tt = 0; tt < nt; ++tt) {
                        const int ro = row0 + tt * tstep;
                        const float ss = net_tile<HT, OUTV, impl::PH_S_FWD>(buf, L.s, L, tab, state, ro);
                        ldj_update(ro, ss, first_in_elem, last_in_elem);
                    }
                }
                impl::ensure_stage(L.t.stage, sg, a);
                const uint8_t* buf = sg.buf();
                for (int tt = 0; tt < nt; ++tt) {
                    const int ro = row0 + tt * tstep;
                    net_tile<HT, OUTV, impl::PH_T_FWD>(buf, L.t, L, tab, state, ro);
                    if (!rnvp) ldj_update(ro, 0.f, first_in_elem, last_in_elem);
                }
            } else {
                impl::ensure_stage(L.t.stage, sg, a);
                const uint8_t* buf = sg.buf();
                for (int tt = 0; tt < nt; ++tt) {
                    const int ro = row0 + tt * tstep;
                    net_tile<HT, OUTV, impl::PH_T_BWD>(buf, L.t, L, tab, state, ro);
                    if (!rnvp) ldj_update(ro, 0.f, first_in_elem, last_in_elem);
                }
                if (rnvp) {
                    impl::ensure_stage(L.s.stage, sg, a);
                    const uint8_t* bs = sg.buf();
                    for (int tt = 0; tt < nt; ++tt) {
                        const int ro = row0 + tt * tstep;
                        const float ss = net_tile<HT, OUTV, impl::PH_S_BWD>(bs, L.s, L, tab, state, ro);
                        ldj_update(ro, -ss, first_in_elem, last_in_elem);  // ln_det_jac = -Σ s
                    }
                }
            }
        }
        have_acc = have_acc || last_in_elem;
    }

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (MODE == MODE_LOGPDF) {
        double part = 0.0;
        if (g == 0) {
            for (int tt = 0; tt < nt; ++tt) {
                const int ro = row0 + tt * tstep;
                const int smp = (wave * nt + tt) * 16 + j;
                float q = 0.f;
                for (int i = 0; i < d; ++i) {
                    const float zz = state[ro + n + i];
                    q = q + zz * zz;
                }
                const float lp = (a.c0 - q / 2.f) + state[ro + cA];
                if (smp < nvalid) {
                    if (a.lp_out) a.lp_out[s0 + smp] = lp;
                    part += (double)lp;
                }
            }
        }
        if (a.partial) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
            __syncthreads();
            double* red = reinterpret_cast<double*>(smem);
            if (lane == 0) red[wave] = part;
            __syncthreads();
            if (tid == 0) {
                double s = 0.0;
                for (int w = 0; w < kWavesPerBlock; ++w) s += red[w];
                a.partial[blockIdx.x] = s;
            }
        }
        if (!a.xout) return;
    }
    __syncthreads();
    for (int i = tid; i < S * d; i += kBlockThreads) {
        const int smp = i / d, c = i - smp * d;
        if (smp < nvalid) a.xout[(s0 + smp) * d + c] = state[smp * stride + n + c];
    }
    if (WANT_LDJ && MODE != MODE_LOGPDF && a.ldj_out) {
        for (int i = tid; i < nvalid; i += kBlockThreads) a.ldj_out[s0 + i] = state[i * stride + cA];
    }
}

template <int HT>
void* uniform_kernel_ptr(int mode, bool outv) {
#define DF_U(M) (outv ? reinterpret_cast<void*>(&uniform_kernel<HT, M, true>) \
                      : reinterpret_cast<void*>(&uniform_kernel<HT, M, false>))
    switch (mode) {
        case MODE_FWD: return DF_U(MODE_FWD);
        case MODE_FWD_INPLACE: return DF_U(MODE_FWD_INPLACE);
        case MODE_BWD: return DF_U(MODE_BWD);
        default: return DF_U(MODE_LOGPDF);
    }
#undef DF_U
}

template <int HT>
hipError_t launch_uniform_ht(int mode, bool outv, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st) {
    void* args[] = {const_cast<ChainArgs*>(&a)};
    return hipLaunchKernel(uniform_kernel_ptr<HT>(mode, outv), dim3(grid), dim3(kBlockThreads), args, lds, st);
}

template <int HT>
hipError_t set_uniform_lds_limit_ht(size_t lds) {
    for (int mode = 0; mode < 4; ++mode)
        for (int ov = 0; ov < 2; ++ov) {
            hipError_t e = hipFuncSetAttribute(uniform_kernel_ptr<HT>(mode, ov != 0),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

template <int HT>
hipError_t uniform_occupancy_ht(int mode, bool outv, size_t lds, int* blocks) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, uniform_kernel_ptr<HT>(mode, outv), kBlockThreads,
                                                        lds);
}

}  // namespace df
