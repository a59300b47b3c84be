// df_small.hip — the small-batch chain kernel.
//
// For a batch that leaves most of the chip idle (config 1 at its stated B = 4096:
// 256 workgroups of 16 samples for 256 CUs) a launch lasts as long as one
// workgroup's dependent chain through the layers.  The specialised kernel's chain is
// long: serial global round trips to copy the tables and the state tile in, LDS round
// trips per feature read, a barrier per stage switch and before the copy-out.  This
// kernel shortens it:
//   * one 16-sample tile per workgroup, on two waves (NW = 2, the default): the
//     s-net of every layer runs on wave 0 and the t-net on wave 1 (the two nets of a
//     layer read the same features, RNVP.jl:174-177, and are independent); wave 1
//     hands its outputs to wave 0 in LDS, wave 0 applies the coupling (RNVP.jl:182-184
//     / 86-90) and keeps the ldj in registers, and a bare barrier (lgkmcnt(0) +
//     s_barrier) after each layer gives wave 1 the updated row.  NW = 1
//     (DF_SMALL_WAVES=1) runs both nets on one wave, no barrier;
//   * the state rows of the tile, vcat(θ, z) plus the zero slot and the 1 of the
//     folded first-Dense bias, sit in a 16 × 13-float LDS patch;
//   * every layer's net fragments are loaded from the blob (the same bytes the LDS
//     stages of the specialised kernel hold) into registers at kernel start, with the
//     rows and the θ bounds, so all loads are in flight before the first use;
//   * the per-layer fields (blob offsets, feature / transformed-dim slots, kinds,
//     element flags, NormalizationLayer bounds) come in a SmallDesc passed by value
//     and held in two VGPRs (v_readlane per field); the θ bounds are read through
//     ChainArgs::tmin / tmax, the chain's device copy.
// The arithmetic is the FAST variant's, operation for operation: the first Dense
// as one f32 MFMA k-step with the bias folded in, the hidden Dense as the
// k-ordered f32 MFMA chain, bias then relu, the output Dense as the VALU GEMV
// reduced over lane groups as ((p0 + p1) + (p2 + p3)) then + b, the coupling
// rounded as z·exp(s), + t (forward) and (x − t), ·exp(−s) (inverse), Σ s in row
// order, the ldj grouped per FlowElement (Blocks.jl:136,149, Chains.jl:160,179) —
// so its outputs are bitwise those of the FAST kernel.  The one difference is the
// order of the fp64 NLL partial sums (one partial per workgroup of 16 samples).
// Phase stamps of the one-wave form: profiles/r04_phase_small_v2.txt.
#include "df_uniform_impl.h"

namespace df {
namespace small {

constexpr int kStride = 13;  // LDS row of a sample: θ | z (n + d <= 8) | zero slot | 2 unused | 1 (folded bias)

struct NetW {      // one FAST hidden-16 net's fragments (the stage layout of df_uniform_impl.h, HT = 1)
    float w0;      // first Dense, KS = 1, bias folded: [lane]
    f32x4 wh;      // hidden 16×16 Dense: [lane][4]
    f32x4 bh;      // hidden bias, rows 4g ..
    f32x4 wo[4];   // output Dense (<= 4 rows): row oo, columns 4g ..
    float bo;      // output bias of lane group g's output (out_valu_t)
};

// A descriptor field as a scalar register.  The per-lane-group selects below would
// otherwise be folded into ONE vector load from the kernel-argument segment at a
// lane-dependent offset — a full memory round trip inside the layer.
template <typename T>
__device__ __forceinline__ T sreg(T v) {
    asm("" : "+s"(v));
    return v;
}

// v[g] for lane group g of four scalar values (register selects)
template <typename T>
__device__ __forceinline__ T by_group(int g, T v0, T v1, T v2, T v3) {
    v0 = sreg(v0);
    v1 = sreg(v1);
    v2 = sreg(v2);
    v3 = sreg(v3);
    return g == 0 ? v0 : g == 1 ? v1 : g == 2 ? v2 : v3;
}

// The descriptor's first 128 dwords in two VGPRs (dword lane and 64 + lane), loaded with
// the rows at kernel start; a layer's fields are then v_readlane's of them.  Read from the
// kernel arguments instead, every field is a scalar load + wait inside the layer (the
// compiler rematerialises them there rather than hold ~100 SGPRs), i.e. a scalar-cache
// round trip per field per layer.
struct DescRegs {
    uint32_t v0, v1;
    __device__ __forceinline__ uint32_t u32(int byte) const {
        const int w = byte >> 2;
        return (uint32_t)__builtin_amdgcn_readlane((int)(w < 64 ? v0 : v1), w & 63);
    }
    __device__ __forceinline__ int i8(int byte) const { return (int)(int8_t)(u32(byte) >> (8 * (byte & 3))); }
    __device__ __forceinline__ float f32(int byte) const { return __uint_as_float(u32(byte)); }
};
#define SD_OFF(f) ((int)offsetof(SmallDesc, f))
static_assert(sizeof(SmallDesc) <= 128 * 4, "DescRegs holds the whole descriptor (128 dwords)");

// net k (0 = s, 1 = t) of layer li: its fragments at the blob offsets of the descriptor
__device__ __forceinline__ void load_net(const ChainArgs& a, const SmallDesc& sd, int li, int k, NetW& w) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    w.w0 = reinterpret_cast<const float*>(a.blob + sd.w0[li][k])[lane];
    w.wh = *reinterpret_cast<const f32x4*>(a.blob + sd.wh[li][k] + lane * 16);
    w.bh = *reinterpret_cast<const f32x4*>(a.blob + sd.wh[li][k] + 1024 + ((4 * g) << 2));
    const uint8_t* w3 = a.blob + sd.wo[li][k];
    const int no = sd.n_out[li];
    // branch-free (one basic block for every net's loads, so they all issue before the
    // first wait): rows past n_out repeat the last one and are never used
#pragma unroll
    for (int oo = 0; oo < 4; ++oo) {
        const int r = oo < no ? oo : (no > 0 ? no - 1 : 0);
        w.wo[oo] = *reinterpret_cast<const f32x4*>(w3 + ((r * 16 + 4 * g) << 2));
    }
    w.bo = reinterpret_cast<const float*>(w3)[no * 16 + (g < no ? g : 0)];
}

// One net on the wave's tile: y = output g of the lane's sample (lane groups g < NO).
// The FAST kernel's functions operation for operation: dense_first (KS = 1, the bias
// folded into k-slot 3), relu, dense_hidden (k-ordered f32 MFMA chain), bias + relu,
// out_valu_t (GEMV, lane-group transpose, + b).
template <int NO>
__device__ __forceinline__ float eval_net(const NetW& w, float xin) {
    f32x4 A = impl::mfma4(w.w0, xin, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int r = 0; r < 4; ++r) A[r] = uni::relu_fast(A[r]);
    f32x4 B = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) B = impl::mfma4(w.wh[r], A[r], B);
    B = B + w.bh;
#pragma unroll
    for (int r = 0; r < 4; ++r) B[r] = uni::relu_fast(B[r]);
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oo = 0; oo < NO; ++oo)
#pragma unroll
        for (int r = 0; r < 4; ++r) p[oo] = __builtin_fmaf(w.wo[oo][r], B[r], p[oo]);
    auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(p[0]), __float_as_uint(p[1]), false, false);
    const float A2 = __uint_as_float(x[0]) + __uint_as_float(x[1]);
    float Bv = 0.f;
    if constexpr (NO > 2) {
        auto y = __builtin_amdgcn_permlane16_swap(__float_as_uint(p[2]), __float_as_uint(p[3]), false, false);
        Bv = __uint_as_float(y[0]) + __uint_as_float(y[1]);
    }
    auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(A2), __float_as_uint(Bv), false, false);
    return (__uint_as_float(c[0]) + __uint_as_float(c[1])) + w.bo;
}

// NW = 2: the s-net of every layer on wave 0 and the t-net on wave 1 of the workgroup
// (the two nets of a layer read the same features, RNVP.jl:174-177, and are
// independent).  Wave 1 hands its outputs over in LDS; wave 0 applies the coupling and
// keeps the ldj; a barrier after each layer gives wave 1 the updated row.  Both waves
// write the initial row (identical values), so a first coupling layer needs no barrier
// (a first NormalizationLayer does: see the kernel).
// Each wave issues one net's instructions per layer instead of two.
// The barriers are bare (lgkmcnt(0) + s_barrier): the LDS row and the handed-over
// outputs are the only data the waves share; no global load needs to land for them.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int MODE, int NL, int NW>
__global__ void __launch_bounds__(64 * NW, 1) small_kernel(ChainArgs a, SmallDesc sd) {
    constexpr bool FWD = (MODE == MODE_FWD || MODE == MODE_FWD_INPLACE);
    constexpr bool WANT_LDJ = (MODE != MODE_FWD_INPLACE);
    __shared__ float srow[16 * kStride];
    __shared__ float yx[NW == 2 ? 64 : 1];  // NW = 2: wave 1's t-net outputs, by lane
    const int wv = NW == 2 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    ClockStamp clk;
    clk.begin(a);
#ifdef DF_PHASE_STAMPS  // diagnostic build (wrong outputs): wave 0 of workgroup 0 stamps its phases
    uint64_t ph[12] = {};
#define DF_PH(i) do { if (blockIdx.x == 0 && wv == 0) ph[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define DF_PH(i) do {} while (0)
#endif
    DF_PH(0);
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
    const int d = a.d, n = a.n, nd = n + d;
    const int64_t smp = (int64_t)blockIdx.x * 16 + j;
    const bool valid = smp < a.batch;
    float* row = srow + j * kStride;

    // every load in flight before the first use: the row (lane group g: columns g, g + 4,
    // g + 8) with the θ bounds of its θ columns (ChainArgs::tmin / tmax, the chain's device
    // copy: a captured train step reads the current bounds), then every coupling net's
    // fragments; branch-free: a clamped address always, the value selected afterwards
    float rv[3], blo[3], bhi[3];
    const int64_t sv = valid ? smp : 0;
    const bool norm_th = a.tmin != nullptr;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int c = g + 4 * q;
        const bool is_th = c < n, is_z = c >= n && c < nd;
        const float* p = is_th ? a.theta + sv * n + c : a.zin + sv * d + (is_z ? c - n : 0);
        const float v = *p;
        rv[q] = ((is_th || is_z) && valid) ? v : (c == nd + 3 ? 1.f : 0.f);
        if (norm_th) {
            const int cb = is_th ? c : 0;
            blo[q] = a.tmin[cb];
            bhi[q] = a.tmax[cb];
        }
    }
    DescRegs dr;
    {
        const uint32_t* sdw = reinterpret_cast<const uint32_t*>(&sd);
        dr.v0 = sdw[lane];
        dr.v1 = sdw[64 + lane];
    }
    // every net's fragments (NormalizationLayers and NICE s-nets load the blob's first
    // bytes, never used: the loads stay one basic block)
    NetW ws[NL], wt[NW == 1 ? NL : 1];  // NW = 2: ws holds this wave's net (s: wave 0, t: wave 1)
#pragma unroll
    for (int li = 0; li < NL; ++li) {
        load_net(a, sd, li, NW == 1 ? 0 : wv, ws[li]);
        if constexpr (NW == 1) load_net(a, sd, li, 1, wt[li]);
    }

#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int c = g + 4 * q;
        float v = rv[q];
        if (c < n && norm_th && valid) {  // normalize_input (Data.jl:213-218)
            const float diff = bhi[q] - blo[q];
            v = (diff == 0.f) ? 0.f : (v - blo[q]) / diff;
        }
        if (c < kStride) row[c] = v;
    }
    // Both waves write the initial row, so a first coupling layer needs no barrier: wave 0
    // writes the row only after the handover barrier inside couple().  A first
    // NormalizationLayer (the inverse pass of a chain that ends with one) is written by
    // wave 0 without that barrier, and wave 1's initial write could land after it and undo
    // it, so that layer waits for both waves' initial writes first.
    if constexpr (NW == 2) {
        if (dr.i8(SD_OFF(kind) + (FWD ? 0 : NL - 1)) == DF_LAYER_NORM) lds_barrier();
    }
    DF_PH(1);
    float ldjA = 0.f, ldjE = 0.f;  // lane group 0: the sample's chain and element ldj
    bool have_acc = false;
    auto ldj_update = [&](float l, bool first_in_elem, bool last_in_elem) {
        const float e = first_in_elem ? l : ldjE + l;
        ldjE = e;
        if (last_in_elem) ldjA = have_acc ? ldjA + e : e;
    };

#pragma unroll
    for (int it = 0; it < NL; ++it) {
        const int li = FWD ? it : NL - 1 - it;
        const int kind = dr.i8(SD_OFF(kind) + li);
        const bool es = dr.i8(SD_OFF(elem_start) + li) != 0, ee = dr.i8(SD_OFF(elem_end) + li) != 0;
        const bool first_in_elem = FWD ? es : ee;
        const bool last_in_elem = FWD ? ee : es;
        if (kind == DF_LAYER_NORM) {  // src/norm/Normalization.jl:64-103
            const float al = dr.f32(SD_OFF(alpha) + 4 * li), be = dr.f32(SD_OFF(beta) + 4 * li), delta = be - al;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int i = g + 4 * q;
                if (i < d) {
                    // lane group g's dims: the bounds by uniform index (register selects)
                    const int x0 = SD_OFF(xmin) + 4 * (8 * li + 4 * q), x1 = SD_OFF(xmax) + 4 * (8 * li + 4 * q);
                    const float lo = by_group(g, dr.f32(x0), dr.f32(x0 + 4), dr.f32(x0 + 8), dr.f32(x0 + 12));
                    const float hi = by_group(g, dr.f32(x1), dr.f32(x1 + 4), dr.f32(x1 + 8), dr.f32(x1 + 12));
                    const float xd = hi - lo;
                    float v = row[n + i];
                    if (FWD) v = ((xd * v - al * hi) + be * lo) / delta;
                    else v = (be * (v - lo) + al * (hi - v)) / xd;
                    if (wv == 0) row[n + i] = v;
                }
            }
            const float lc = dr.f32(SD_OFF(ldj_const) + 4 * li);
            ldj_update(FWD ? lc : -lc, first_in_elem, last_in_elem);
        } else {
            const bool rnvp = (kind == DF_LAYER_RNVP);
            // byte g of the layer's feature / transformed-dim words (slots < 13: unsigned)
            const int fslot = (int)((dr.u32(SD_OFF(feat) + 4 * li) >> (8 * g)) & 0xffu);
            const float xin = row[fslot];
            const int slot = (int)((dr.u32(SD_OFF(af) + 4 * li) >> (8 * g)) & 0xffu);
            auto couple = [&](auto no_tag) {
                constexpr int NO = decltype(no_tag)::value;
                float ys, yt;
                if constexpr (NW == 1) {
                    ys = rnvp ? eval_net<NO>(ws[li], xin) : 0.f;
                    yt = eval_net<NO>(wt[li], xin);
                } else {
                    const float y = (wv == 1 || rnvp) ? eval_net<NO>(ws[li], xin) : 0.f;
                    if (wv == 1) yx[lane] = y;
                    lds_barrier();
                    if (wv == 1) return;
                    ys = y;
                    yt = yx[lane];
                }
                if (g < NO) {
                    float v = row[slot];
                    if (FWD) {
                        if (rnvp) v = v * expf(ys);
                        v = v + yt;
                    } else {
                        v = v - yt;
                        if (rnvp) v = v * expf(-ys);
                    }
                    row[slot] = v;
                }
                // ldj = Σ_k s_k in row order (RNVP.jl:180 / :86), valid in lane group 0
                const float sum = rnvp ? uni::group_row_sum<NO>(ys) : 0.f;
                ldj_update(rnvp ? (FWD ? sum : -sum) : 0.f, first_in_elem, last_in_elem);
            };
            switch (dr.i8(SD_OFF(n_out) + li)) {
                case 1: couple(std::integral_constant<int, 1>{}); break;
                case 2: couple(std::integral_constant<int, 2>{}); break;
                case 3: couple(std::integral_constant<int, 3>{}); break;
                default: couple(std::integral_constant<int, 4>{}); break;
            }
        }
        have_acc = have_acc || last_in_elem;
        DF_PH(2 + it);
        if constexpr (NW == 2) {
            lds_barrier();  // wave 0's row update → wave 1's next features
        }
        if (!FWD && a.snap && valid && wv == 0) {  // training: every layer's output for the reverse sweep
            float* dst = a.snap + (int64_t)li * a.batch * d;
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (g + 4 * q < d) dst[smp * d + g + 4 * q] = row[n + g + 4 * q];
        }
    }

    if (NW == 2 && wv == 1) return;  // wave 0 holds the ldj and writes every output
    if (MODE == MODE_LOGPDF) {
        double part = 0.0;
        if (g == 0) {
            float q = 0.f;
            for (int i = 0; i < d; ++i) {
                const float zz = row[n + i];
                q = q + zz * zz;
            }
            const float lp = (a.c0 - q / 2.f) + ldjA;
            if (valid) {
                if (a.lp_out) a.lp_out[smp] = lp;
                part = (double)lp;
            }
        }
        if (a.partial) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
            if (lane == 0) a.partial[blockIdx.x] = part;
        }
        if (!a.xout) {
            clk.end(a);
            return;
        }
    }
    if (valid) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (g + 4 * q < d) a.xout[smp * d + g + 4 * q] = row[n + g + 4 * q];
        if (WANT_LDJ && MODE != MODE_LOGPDF && a.ldj_out && g == 0) a.ldj_out[smp] = ldjA;
    }
#ifdef DF_PHASE_STAMPS
    DF_PH(6);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DF_PH(7);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < 8; ++i) a.xout[i] = (float)(ph[i] - ph[0]);
    }
#endif
#undef DF_PH
    clk.end(a);
}

template <int MODE, int NW>
void* kernel_ptr_m(int nl) {
    switch (nl) {
        case 1: return reinterpret_cast<void*>(&small_kernel<MODE, 1, NW>);
        case 2: return reinterpret_cast<void*>(&small_kernel<MODE, 2, NW>);
        case 3: return reinterpret_cast<void*>(&small_kernel<MODE, 3, NW>);
        case 4: return reinterpret_cast<void*>(&small_kernel<MODE, 4, NW>);
        default: return nullptr;
    }
}

template <int NW>
void* kernel_ptr_w(int mode, int nl) {
    switch (mode) {
        case MODE_FWD: return kernel_ptr_m<MODE_FWD, NW>(nl);
        case MODE_FWD_INPLACE: return kernel_ptr_m<MODE_FWD_INPLACE, NW>(nl);
        case MODE_BWD: return kernel_ptr_m<MODE_BWD, NW>(nl);
        default: return kernel_ptr_m<MODE_LOGPDF, NW>(nl);
    }
}

void* kernel_ptr(int mode, int nl, int nw) { return nw == 2 ? kernel_ptr_w<2>(mode, nl) : kernel_ptr_w<1>(mode, nl); }

}  // namespace small

hipError_t launch_small(int mode, const ChainArgs& a, const SmallDesc& sd, unsigned grid, hipStream_t st, int nw) {
    nw = nw == 1 ? 1 : 2;
    void* f = small::kernel_ptr(mode, a.n_layers, nw);
    if (!f) return hipErrorInvalidValue;
    void* args[] = {const_cast<ChainArgs*>(&a), const_cast<SmallDesc*>(&sd)};
    return hipLaunchKernel(f, dim3(grid), dim3(64 * nw), args, 0, st);
}

}  // namespace df
