// df_train_impl.h — the reverse-sweep kernel of one conditioner net.
//
// Every wave owns 16-sample tiles (persistent grid); a SPLIT instance's wave carries
// kTrainSplitTT of them through every step together (df_train.h: one wave per SIMD,
// two independent chains per wave).  Per tile:
//   forward recompute   x → A0 = σ0(W0 x + b0) [→ A1 = σh(W1 A0 + b1)] → y = σo(W3 h + b3)
//                       (same device functions and rounding as the inverse
//                       pass, so s and t are bitwise those of step 1);
//   coupling pullback   s-net: s̄ = -z̄_af·z_af + 1/N (z_af = U[li]_af; j̄ = -1/N)
//                       t-net: t̄ = -z̄_af·exp(-s)  (NICE: t̄ = -z̄_af),
//                              then ū_af = z̄_af·exp(-s)   src/affine/RNVP.jl:133-139
//   Dense backward      δ = ȳ ⊙ σ'(y);  dW += δ·inᵀ,  db += Σ δ;  in̄ = Wᵀ δ.
// Wᵀδ chains on MFMA exactly like the forward pass (transposed fragments,
// accumulator = next B operand).  dW = δ·inᵀ contracts over samples, which
// sit on lanes 0..15 of the accumulator layout: both operands go through a
// per-wave LDS transpose T[row][sample] and are read back as f32x4 fragments
// (k-step s of lane group g uses sample 4g + s).  dW / db accumulate in
// registers over all of a wave's tiles; the 8 waves are summed in LDS in a
// fixed order and each workgroup writes its partial (no atomics: the final
// reduction over workgroups is a separate fixed-order kernel, so gradients
// are bitwise reproducible).
// The conditioner input gradient is added to z̄ of the identity dims.
#pragma once

#include "df_train.h"
#include "df_uniform_impl.h"

namespace df {
namespace trn {

using impl::mfma4;

__device__ __forceinline__ f32x4 lds4f(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// σ'(x) from y = σ(x): NNlib's derivative table (src/activations.jl, UNARY_ACTS)
// for the activations whose rule is written in Ω alone.
__device__ __forceinline__ float act_grad(int act, float y) {
    switch (act) {
        case DF_ACT_RELU: return y > 0.f ? 1.f : 0.f;
        case DF_ACT_TANH: return 1.f - y * y;                     // tanh_fast: 1 - Ω²
        case DF_ACT_SIGMOID: return y * (1.f - y);                // sigmoid_fast: Ω(1 - Ω)
        case DF_ACT_LEAKYRELU: return y > 0.f ? 1.f : 0.01f;      // ifelse(Ω > 0, 1, 1//100)
        case DF_ACT_ELU: return y >= 0.f ? 1.f : y + 1.f;         // deriv_elu(Ω) = ifelse(Ω ≥ 0, 1, Ω + α)
        case kDactStored: return y;
        default: return 1.f;
    }
}

__device__ __forceinline__ bool act_needs_pre(int act) {
    return act == DF_ACT_SOFTPLUS || act == DF_ACT_LOGCOSH || act == DF_ACT_SWISH;
}

// σ'(x) from the pre-activation x and y = σ(x) (NNlib: softplus → sigmoid_fast(x),
// logcosh → tanh(x), swish → Ω + sigmoid_fast(x)·(1 − Ω)); the rest as act_grad.
__device__ __forceinline__ float act_dx(int act, float x, float y) {
    switch (act) {
        case DF_ACT_SOFTPLUS: return impl::sigmoid_fast(x);
        case DF_ACT_LOGCOSH: return tanhf(x);
        case DF_ACT_SWISH: return y + impl::sigmoid_fast(x) * (1.f - y);
        default: return act_grad(act, y);
    }
}

// v = σ.(v) in place, σ'(pre) into dv (AM_PRE recompute)
template <int HT>
__device__ __forceinline__ void act_keep_grad(int act, f32x4 (&v)[HT], f32x4 (&dv)[HT]) {
#pragma unroll
    for (int m = 0; m < HT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float x = v[m][r];
            const float y = (act == DF_ACT_IDENTITY) ? x : impl::act_fn(act, x);
            dv[m][r] = act_dx(act, x, y);
            v[m][r] = y;
        }
}

template <int HT, bool RELU>
__device__ __forceinline__ void mul_act_grad(int act, const f32x4 (&y)[HT], f32x4 (&gr)[HT]) {
    if (RELU || act == DF_ACT_RELU) {
#pragma unroll
        for (int m = 0; m < HT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) gr[m][r] = (y[m][r] > 0.f) ? gr[m][r] : 0.f;
    } else if (act != DF_ACT_IDENTITY) {
#pragma unroll
        for (int m = 0; m < HT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) gr[m][r] = gr[m][r] * act_grad(act, y[m][r]);
    }
}

// Column-quad swizzle of the transpose buffers: quad q of row R is stored at quad
// q ^ rswz(R), rswz(R) = the Gray bit of (R >> 2) & 3 (0, 1, 1, 0) ^ bit 4 of R.  With
// the 20-float rows, both b128 read shapes, (row 16m + j, quad g) and the M4 operands'
// (row lane, quad q), land on 16 distinct 4-bank groups in every 16-lane group of
// ds_read_b128 (a search over row swizzles; the Gray bit alone leaves the
// second shape 2-way); the b32 row writes keep their bank sets (a permutation inside
// the row).
__device__ __forceinline__ int tswz(int q) { return DF_TRAIN_SWZ ? ((q ^ (q >> 1)) & 1) : 0; }
__device__ __forceinline__ int rswz(int row) { return DF_TRAIN_SWZ ? (tswz(row >> 2) ^ ((row >> 4) & 1)) : 0; }
// element (row, col) of a transpose buffer
__device__ __forceinline__ int tidx(int row, int col) {
    return row * kTS + ((((col >> 2) ^ rswz(row)) << 2) | (col & 3));
}
// f32x4 fragment (row, quad q) of a transpose buffer
__device__ __forceinline__ f32x4 tread(const float* T, int row, int q) {
    return *reinterpret_cast<const f32x4*>(T + row * kTS + ((q ^ rswz(row)) << 2));
}

// accumulator-layout tile (rows 16m + 4g + r of sample j) → T[row][j]; the row's
// quad swizzle is tswz(g) ^ (m & 1) for every r, so the lane's column is fixed per m
template <int HT>
__device__ __forceinline__ void t_write(float* T, const f32x4 (&v)[HT]) {
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
#pragma unroll
    for (int m = 0; m < HT; ++m) {
        const int col = (((j >> 2) ^ (DF_TRAIN_SWZ ? tswz(g) ^ (m & 1) : 0)) << 2) | (j & 3);
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(16 * m + 4 * g + r) * kTS + col] = v[m][r];
    }
}

// Scalar f32 adds the compiler cannot pair into v_pk_add_f32: a packed f32 add issues at a
// quarter of v_add_f32's rate (tools/probe/mfma_pair.hip) and its operand pairs cost moves.
// Same operations in the same order as the plain expressions.
__device__ __forceinline__ float fadd(float a, float b) {
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float hsum4(f32x4 v) { return fadd(fadd(v[0], v[1]), fadd(v[2], v[3])); }

__device__ __forceinline__ void lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

}  // namespace trn

// bf16x4 halves of the SPLIT dW1 operands (4 samples of one row, one plane)
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split4(f32x4 v, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
#pragma unroll
    for (int e = 0; e < 4; e += 2) {
        uni::bf16x2 h, m, l;
        uni::split2(v[e], v[e + 1], h, m, l);
        p0[e] = h[0]; p0[e + 1] = h[1];
        p1[e] = m[0]; p1[e + 1] = m[1];
        p2[e] = l[0]; p2[e + 1] = l[1];
    }
}

__device__ __forceinline__ uni::bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// The three planes of 4 values as one run [p1 p0 p2] (DF_TRAIN_DW1_CONTIG): both SPLIT
// dW1 operands of a row tile are 4-dword windows of it.
#ifndef DF_TRAIN_DW1_CONTIG
#define DF_TRAIN_DW1_CONTIG 1
#endif
typedef __bf16 bf16x12 __attribute__((ext_vector_type(12)));

__device__ __forceinline__ bf16x12 split4_run(f32x4 v) {
    bf16x12 q;
#pragma unroll
    for (int e = 0; e < 4; e += 2) {
        uni::bf16x2 h, m, l;
        uni::split2(v[e], v[e + 1], h, m, l);
        q[e] = m[0]; q[e + 1] = m[1];
        q[4 + e] = h[0]; q[5 + e] = h[1];
        q[8 + e] = l[0]; q[9 + e] = l[1];
    }
    return q;
}
__device__ __forceinline__ uni::bf16x8 run_lo(const bf16x12& q) {  // [p1 | p0]
    return __builtin_shufflevector(q, q, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ uni::bf16x8 run_hi(const bf16x12& q) {  // [p0 | p2]
    return __builtin_shufflevector(q, q, 4, 5, 6, 7, 8, 9, 10, 11);
}

// dW_out and dW0 of the SPLIT instances (one first-Dense k-step: <= 4 features, <= 4
// outputs) on v_mfma_f32_4x4x1_16b_f32: 16 blocks of 4×4, one sample per instruction,
// block b = lane / 4 owning hidden rows 4b..4b+3 — no zero-padded rows (the 16x16x4
// form spends 12 of its 16 rows on padding there).  Lane l then holds dW_out[0..3][l]
// and dW0[4(l/4) + 0..3][l % 4].
#ifndef DF_TRAIN_M4
#define DF_TRAIN_M4 1
#endif
__device__ __forceinline__ f32x4 mfma4x4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

// NAF > 0: the transformed-dim count (= output count) at compile time (SPLIT instances,
// 2 and 3: the d = 5 chains; the launcher also requires ≤ 4 conditioner inputs);
// 0: a.n_af at run time.
template <int HT, int NH, int AM, bool SPLIT = false, int NAF = 0>
__global__ void __launch_bounds__(train_threads(SPLIT), 1) train_net_kernel(TrainArgs a) {
    using namespace trn;
    const int n_af = NAF > 0 ? NAF : a.n_af;
    constexpr bool RELU = (AM == AM_RELU);
    constexpr bool PRE = (AM == AM_PRE);
    constexpr bool M4 = SPLIT && DF_TRAIN_M4;
    // tiles per wave (df_train.h kTrainSplitTT): every per-tile step below runs over the TT
    // tiles back to back, so one wave issues two independent chains
    constexpr int TT = SPLIT ? kTrainSplitTT : 1;
    constexpr int NW = kTrainWaves / TT, NT = 64 * NW;  // waves, threads per workgroup
    static_assert(!SPLIT || (RELU && NH == 1 && HT >= 2), "SPLIT: relu nets with one hidden Dense, hidden 32/64");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const GNet& G = a.net;
    const UNet& N = SPLIT ? G.su : G.u;
    const int fwd_bytes = SPLIT ? G.sfwd_bytes : G.fwd_bytes;
    const int t_bytes = SPLIT ? HT * 1024 : G.t_bytes;  // SPLIT: W0ᵀ only (W1ᵀ as planes)
    uint8_t* fw = smem;
    uint8_t* tw = smem + fwd_bytes;
    uint8_t* stw = tw + t_bytes;
    float* tarea = reinterpret_cast<float*>(stw + (SPLIT ? G.st_bytes : 0));

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, j = lane & 15;
    const int d = a.d, n = a.n;
    constexpr int TROWS = 16 * HT;
    constexpr int INP = 16 * HT;
    // transpose buffers of tile t of this wave: TA(t) (δ side), TB(t) (activation side)
    float* const TW = tarea + wave * TT * 2 * TROWS * kTS;
    auto TA = [&](int t) { return TW + t * 2 * TROWS * kTS; };
    auto TB = [&](int t) { return TW + t * 2 * TROWS * kTS + TROWS * kTS; };
    const bool sph = (a.phase == TR_PHASE_S);
    const bool rnvp = (a.kind == DF_LAYER_RNVP);

    {  // the net's forward and transposed fragments → LDS
        const f32x4* src = reinterpret_cast<const f32x4*>(SPLIT ? a.sblob + G.sfwd_src : a.blob + G.fwd_src);
        for (int i = tid; i < fwd_bytes / 16; i += NT) reinterpret_cast<f32x4*>(fw)[i] = src[i];
        const f32x4* srt = reinterpret_cast<const f32x4*>(a.tblob + G.t_src);
        if constexpr (NAF > 0) {
            // W0ᵀ alone (SPLIT), read only by the 4x4x1 x̄, which takes the fragments of lanes
            // (lane & 3) + 16g: those 16 per k-quad go to slots (lane & 3) + 4g, one 256-byte
            // run (its ds_read_b128 then hit 16 distinct bank groups instead of 4)
            const int w0 = G.off_w0t / 16;
            for (int i = tid; i < HT * 16; i += NT) {
                const int kq = i >> 4, c = i & 15;
                reinterpret_cast<f32x4*>(tw)[w0 + kq * 64 + c] = srt[w0 + kq * 64 + (c & 3) + 16 * (c >> 2)];
            }
        } else {
            for (int i = tid; i < t_bytes / 16; i += NT) reinterpret_cast<f32x4*>(tw)[i] = srt[i];
        }
        if constexpr (SPLIT) {
            const f32x4* sst = reinterpret_cast<const f32x4*>(a.tsblob + G.st_src);
            for (int i = tid; i < G.st_bytes / 16; i += NT) reinterpret_cast<f32x4*>(stw)[i] = sst[i];
        }
    }
    // zero rows of the δ_out transposes that no lane writes (rows >= 4)
#pragma unroll
    for (int t = 0; t < TT; ++t)
        for (int i = lane; i < TROWS * kTS; i += 64) TA(t)[i] = 0.f;
    __syncthreads();

    // h̄ = W_outᵀ ȳ on the matrix pipe (DF_TRAIN_HB_MFMA; the SPLIT instances with the
    // output count at compile time): A = W_out[g][16m + j] (a loop-invariant float per row
    // tile, 0 for g >= n_af), B = ȳ[g] of sample j — the k = 4 slots are the ≤ 4 outputs
#ifndef DF_TRAIN_HB_MFMA
#define DF_TRAIN_HB_MFMA 1
#endif
    constexpr bool HBM = SPLIT && NAF > 0 && DF_TRAIN_HB_MFMA;
    float w3a[HT];
#pragma unroll
    for (int m = 0; m < HT; ++m)
        w3a[m] = (HBM && g < n_af) ? reinterpret_cast<const float*>(fw + N.off_out)[g * INP + 16 * m + j] : 0.f;
    constexpr int NHT = NH ? HT : 1;
    f32x4 gW0[HT], gWo[HT], gWh[NHT][NHT];
    float gb0[HT], gbh[NHT], gbo = 0.f;
    f32x4 gWo4 = f32x4{0.f, 0.f, 0.f, 0.f}, gW04 = f32x4{0.f, 0.f, 0.f, 0.f};  // M4 accumulators
    float gb0l = 0.f;                                                          // M4: Σ δ0[lane]
    const int lrow = lane < TROWS ? lane : TROWS - 1;  // M4 operand row of this lane (clamped)
#pragma unroll
    for (int m = 0; m < HT; ++m) {
        gW0[m] = gWo[m] = f32x4{0.f, 0.f, 0.f, 0.f};
        gb0[m] = 0.f;
    }
#pragma unroll
    for (int m = 0; m < NHT; ++m) {
        gbh[m] = 0.f;
#pragma unroll
        for (int q = 0; q < NHT; ++q) gWh[m][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // Loop-invariant gather tables of this lane (no dependent table loads per tile):
    // conditioner feature k = 4r + g of vcat(θ, u)[axis_nn] (kind 0 zero, 1 θ, 2 u,
    // 3 the folded bias's 1), the x̄ targets f = 4g + r (z̄ columns of identity dims,
    // -1 otherwise) and the transformed dims (z̄ columns).
    // Packed: xcode[r] = kind << 8 | offset; zxp8 / afp8 one byte per r (0xff: none).
    int xcode[4];
    uint32_t zxp8 = 0, afp8 = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        xcode[r] = 0;
        if (r < N.ks) {
            const int slot = a.feat[4 * r + g];
            if (slot < n) xcode[r] = 1 << 8 | slot;
            else if (slot < n + d) xcode[r] = 2 << 8 | (slot - n);
            else if (slot == n + d + 3) xcode[r] = 3 << 8;  // folded first-Dense bias (df_plan.cpp pass 1c)
        }
        const int f = 4 * g + r;
        const int fs = (f < G.n_in) ? a.feat[f] : -1;
        zxp8 |= (uint32_t)((fs >= n && fs < n + d) ? fs - n : 0xff) << (8 * r);
        afp8 |= (uint32_t)((r < n_af) ? a.af[r] - n : 0xff) << (8 * r);
    }
    // per-iteration opaque copies of the tables (refreshed at each tile start): the
    // compiler must not hoist 64-bit addresses derived from them out of the tile loop
    // (a dozen pointers held live across the loop spill the accumulators)
    uint32_t zxl = zxp8, afl = afp8;
    int xcl[4] = {xcode[0], xcode[1], xcode[2], xcode[3]};
    auto zxc = [&](int r) { return (int)((zxl >> (8 * r)) & 0xffu); };
    auto afc = [&](int r) { return (int)((afl >> (8 * r)) & 0xffu); };
    // A tile's global inputs, each issued ahead of its use with independent
    // addresses (one memory latency, covered by the MFMA work between issue and use):
    // raw features at the tile start; z̄ of the transformed dims and u_out of those
    // dims (s phase) or exp(-s) (t phase) before the hidden Dense; z̄ of the x̄
    // targets before W1ᵀδ.
    auto load_x = [&](int64_t s, bool ok, float (&xr)[4]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int kind = xcl[r] >> 8, off = xcl[r] & 0xff;
            xr[r] = 0.f;
            if (ok && kind == 1) xr[r] = a.theta[s * n + off];
            if (ok && kind == 2) xr[r] = a.u_in[s * d + off];
        }
    };
    auto load_pull = [&](int64_t s, bool ok, float (&zbv)[4], float (&aux)[4]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            zbv[r] = (ok && afc(r) != 0xff) ? a.zbar[s * d + afc(r)] : 0.f;
            aux[r] = 1.f;
            if (ok && afc(r) != 0xff) {
                if (sph) aux[r] = a.u_out[s * d + afc(r)];
                else if (rnvp) aux[r] = a.ebuf[s * 4 + r];
            }
        }
    };
    auto load_zx = [&](int64_t s, bool ok, float (&zxv)[4]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) zxv[r] = (ok && zxc(r) != 0xff) ? a.zbar[s * d + zxc(r)] : 0.f;
    };

    // wave-tile-group p holds the TT consecutive tiles TT·p .. TT·p + TT − 1
    const int64_t ntiles = (a.batch + 15) / 16;
    const int64_t pstride = (int64_t)gridDim.x * NW;
    for (int64_t p = (int64_t)blockIdx.x * NW + wave; p * TT < ntiles; p += pstride) {
        int64_t s[TT];
        bool valid[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            s[t] = (p * TT + t) * 16 + j;
            valid[t] = s[t] < a.batch;
        }
        zxl = zxp8;
        afl = afp8;
        asm volatile("" : "+v"(zxl), "+v"(afl));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            xcl[r] = xcode[r];
            asm volatile("" : "+v"(xcl[r]));
        }
        float xr[TT][4], zbp[TT][4], aux[TT][4], zxp[TT][4];
#pragma unroll
        for (int t = 0; t < TT; ++t) load_x(s[t], valid[t], xr[t]);

        // ---- conditioner input, features k = 4r + g of vcat(θ, u)[axis_nn] ----
        float xin[TT][4];
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = xr[t][r];
                const int kind = xcl[r] >> 8;
                if (kind == 1 && a.tmin) {  // normalize_input (Data.jl:213-218)
                    const int slot = xcl[r] & 0xff;
                    const float lo = a.tmin[slot], diff = a.tmax[slot] - lo;
                    v = (diff == 0.f) ? 0.f : (v - lo) / diff;
                }
                if (kind == 3) v = 1.f;
                xin[t][r] = valid[t] ? v : 0.f;
            }

        // ---- forward recompute ----
        f32x4 A0[TT][HT], A1[TT][HT];
        constexpr int NP = PRE ? HT : 1;
        f32x4 D0[NP], D1[NP];  // AM_PRE (TT = 1): σ'(pre) of the first / hidden Dense
        if constexpr (SPLIT) {  // the inverse pass's SPLIT kernel functions: bitwise its s and t
            uni::dense_first_split<HT, TT>(fw, N, xin, A0);
            uni::bias_act<HT, TT, true>(fw, DF_ACT_RELU, A0, false);
        } else {
            uni::dense_first<HT, TT>(fw, N, xin, A0);
        }
        if constexpr (SPLIT) {
        } else if constexpr (PRE) {
            uni::bias_act<HT, TT, false>(fw + N.off_b0, DF_ACT_IDENTITY, A0, !N.fold0);
            act_keep_grad<HT>(N.act0, A0[0], D0);
        } else {
            uni::bias_act<HT, TT, RELU>(fw + N.off_b0, N.act0, A0, !N.fold0);
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) load_pull(s[t], valid[t], zbp[t], aux[t]);
        if constexpr (SPLIT) {
            uni::dense_hidden_split<HT, TT, true, true>(fw + N.off_h, A0, A1);
            uni::bias_act<HT, TT, true>(fw, DF_ACT_RELU, A1, false);
        } else if constexpr (NH == 1) {
            uni::dense_hidden<HT, TT>(fw + N.off_h, A0, A1);
            if constexpr (PRE) {
                uni::bias_act<HT, TT, false>(fw + N.off_h + HT * HT * 1024, DF_ACT_IDENTITY, A1);
                act_keep_grad<HT>(N.acth, A1[0], D1);
            } else {
                uni::bias_act<HT, TT, RELU>(fw + N.off_h + HT * HT * 1024, N.acth, A1);
            }
        }
        const f32x4(&H)[TT][HT] = NH ? A1 : A0;
        f32x4 o[TT];
        float dfo[4] = {1.f, 1.f, 1.f, 1.f};  // AM_PRE: σo'(pre) of the output Dense
        if constexpr (PRE) {
            uni::out_valu<HT, TT, true, NAF>(fw, N, H, o);  // pre-activation (no σo)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float x = o[0][k];
                const float y = (N.act_out == DF_ACT_IDENTITY) ? x : impl::act_fn(N.act_out, x);
                dfo[k] = act_dx(N.act_out, x, y);
                o[0][k] = y;
            }
        } else {
            uni::out_valu<HT, TT, RELU, NAF>(fw, N, H, o);
        }

        // ---- coupling pullback → ȳ (every lane group holds all outputs of sample j) ----
        float dout[TT][4], zb[TT][4], ee[TT][4];
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                dout[t][k] = 0.f;
                zb[t][k] = 0.f;
                ee[t][k] = 1.f;
                if (k < n_af && valid[t]) {
                    zb[t][k] = zbp[t][k];
                    if (sph) {
                        ee[t][k] = expf(-o[t][k]);
                        dout[t][k] = -zb[t][k] * aux[t][k] + a.inv_n;  // s̄ = -z̄_af·z_af - j̄
                    } else {
                        if (rnvp) ee[t][k] = aux[t][k];
                        dout[t][k] = -zb[t][k] * ee[t][k];             // t̄ = -z̄_af·exp(-s)
                    }
                    if (PRE) {
                        if (N.act_out != DF_ACT_IDENTITY) dout[t][k] = dout[t][k] * dfo[k];
                    } else if (!RELU && N.act_out != DF_ACT_IDENTITY) {
                        dout[t][k] = dout[t][k] * act_grad(N.act_out, o[t][k]);
                    }
                }
            }
#pragma unroll
        for (int t = 0; t < TT; ++t)
            if (sph && g == 0 && valid[t]) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < n_af) a.ebuf[s[t] * 4 + k] = ee[t][k];
            }

        // ---- output Dense: dW3 += ȳ·hᵀ, db3 += Σȳ, h̄ = W3ᵀ ȳ ----
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if (g == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) TA(t)[tidx(r, j)] = dout[t][r];
            }
            t_write<HT>(TB(t), H[t]);
        }
        lds_order();
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if constexpr (M4) {  // block b: A = ȳ[lane % 4][s], B = h[lane][s], one sample s per step
                const f32x4 fa = tread(TA(t), j, g);
                gbo = fadd(gbo, hsum4(fa));
                f32x4 yv[4], hv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    yv[q] = tread(TA(t), lane & 3, q);
                    hv[q] = tread(TB(t), lrow, q);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) gWo4 = mfma4x4(yv[q][e], hv[q][e], gWo4);
            } else {
                const f32x4 fa = tread(TA(t), j, g);
                gbo = fadd(gbo, hsum4(fa));
#pragma unroll
                for (int mb = 0; mb < HT; ++mb) {
                    const f32x4 fb = tread(TB(t), 16 * mb + j, g);
#pragma unroll
                    for (int q = 0; q < 4; ++q) gWo[mb] = mfma4(fa[q], fb[q], gWo[mb]);
                }
            }
        }
        f32x4 hb[TT][HT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if constexpr (HBM) {  // one v_mfma_f32_16x16x4_f32 per row tile: k = output g of sample j
                const float bk = g == 0 ? dout[t][0] : g == 1 ? dout[t][1] : g == 2 ? dout[t][2] : dout[t][3];
#pragma unroll
                for (int m = 0; m < HT; ++m) hb[t][m] = mfma4(w3a[m], bk, f32x4{0.f, 0.f, 0.f, 0.f});
            } else {
#pragma unroll
            for (int m = 0; m < HT; ++m) hb[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k < n_af) {
#pragma unroll
                    for (int m = 0; m < HT; ++m) {
                        const f32x4 w = impl::lds4(fw + N.off_out + ((k * INP + 16 * m + 4 * g) << 2));
                        hb[t][m] = hb[t][m] + w * dout[t][k];
                    }
                }
            }
            }
            if constexpr (PRE) {
                const f32x4(&DH)[NP] = NH ? D1 : D0;
#pragma unroll
                for (int m = 0; m < HT; ++m) hb[t][m] = hb[t][m] * DH[m];
            } else {
                mul_act_grad<HT, RELU>(NH ? N.acth : N.act0, H[t], hb[t]);
            }
        }

        // ---- hidden Dense: dW1 += δ·A0ᵀ, db1 += Σδ, Ā0 = W1ᵀ δ ----
        f32x4 d0[TT][HT];
        if constexpr (NH == 1) {
            lds_order();
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                t_write<HT>(TA(t), hb[t]);
                t_write<HT>(TB(t), A0[t]);
            }
            lds_order();
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                f32x4 fa[HT], fb[HT];
#pragma unroll
                for (int m = 0; m < HT; ++m) {
                    fa[m] = tread(TA(t), 16 * m + j, g);
                    fb[m] = tread(TB(t), 16 * m + j, g);
                    gbh[m] = fadd(gbh[m], hsum4(fa[m]));
                }
                if constexpr (SPLIT && DF_TRAIN_DW1_CONTIG) {
                    // Planes of 4 samples in one 6-dword run per row tile, [p1 p0 p2]: its
                    // dwords 0-3 ([p1|p0]) and 2-5 ([p0|p2]) are the MFMA operands, no
                    // operand assembly.  k-slot (g, e): sample 4g + (e & 3), plane pair
                    // e >> 2; small terms first:  δ[p0|p2]·A0[p1|p0] = δ0·a1 + δ2·a0,
                    // δ[p1|p0]·A0[p0|p2] = δ1·a0 + δ0·a2,  δ[p1|p0]·A0[p1|p0] = δ1·a1 + δ0·a0.
                    bf16x12 qb[HT];
#pragma unroll
                    for (int m = 0; m < HT; ++m) qb[m] = split4_run(fb[m]);
#pragma unroll
                    for (int ma = 0; ma < HT; ++ma) {
                        const bf16x12 qa = split4_run(fa[ma]);
                        const uni::bf16x8 a_lo = run_lo(qa), a_hi = run_hi(qa);
#pragma unroll
                        for (int mb = 0; mb < HT; ++mb) {
                            const uni::bf16x8 b_lo = run_lo(qb[mb]), b_hi = run_hi(qb[mb]);
                            f32x4 v = gWh[ma][mb];
                            v = uni::mfma_bf(a_hi, b_lo, v);
                            v = uni::mfma_bf(a_lo, b_hi, v);
                            gWh[ma][mb] = uni::mfma_bf(a_lo, b_lo, v);
                        }
                    }
                } else if constexpr (SPLIT) {
                    // k-slot (g, e) of MFMA u: sample 4g + (e & 3), product 2u + (e >> 2) of
                    // (w0x0, w0x1 | w1x0, w0x2 | w1x1, w2x0), δ rows as A, A0 rows as B
                    bf16x4 pb[HT][3];
#pragma unroll
                    for (int m = 0; m < HT; ++m) split4(fb[m], pb[m][0], pb[m][1], pb[m][2]);
#pragma unroll
                    for (int ma = 0; ma < HT; ++ma) {
                        bf16x4 pa[3];
                        split4(fa[ma], pa[0], pa[1], pa[2]);
                        const uni::bf16x8 a0 = cat8(pa[1], pa[2]), a1 = cat8(pa[1], pa[0]), a2 = cat8(pa[0], pa[0]);
#pragma unroll
                        for (int mb = 0; mb < HT; ++mb) {  // small terms first
                            f32x4 v = gWh[ma][mb];
                            v = uni::mfma_bf(a0, cat8(pb[mb][1], pb[mb][0]), v);
                            v = uni::mfma_bf(a1, cat8(pb[mb][0], pb[mb][2]), v);
                            gWh[ma][mb] = uni::mfma_bf(a2, cat8(pb[mb][0], pb[mb][1]), v);
                        }
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int ma = 0; ma < HT; ++ma)
#pragma unroll
                            for (int mb = 0; mb < HT; ++mb) gWh[ma][mb] = mfma4(fa[ma][q], fb[mb][q], gWh[ma][mb]);
                }
            }
#pragma unroll
            for (int t = 0; t < TT; ++t) load_zx(s[t], valid[t], zxp[t]);
            if constexpr (SPLIT) uni::dense_hidden_split<HT, TT, false, true>(stw, hb, d0);
            else uni::dense_hidden<HT, TT>(tw + G.off_ht, hb, d0);
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                if constexpr (PRE) {
#pragma unroll
                    for (int m = 0; m < HT; ++m) d0[t][m] = d0[t][m] * D0[m];
                } else {
                    mul_act_grad<HT, RELU>(N.act0, A0[t], d0[t]);
                }
            }
        } else {
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                load_zx(s[t], valid[t], zxp[t]);
#pragma unroll
                for (int m = 0; m < HT; ++m) d0[t][m] = hb[t][m];
            }
        }

        // ---- first Dense: dW0 += δ0·xᵀ, db0 += Σδ0, x̄ = W0ᵀ δ0 ----
        lds_order();
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            t_write<HT>(TA(t), d0[t]);
#pragma unroll
            for (int r = 0; r < 4; ++r) TB(t)[tidx(4 * r + g, j)] = xin[t][r];
        }
        lds_order();
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if constexpr (M4) {  // block b: A = δ0[lane][s], B = x[lane % 4][s]
                f32x4 dv[4], xv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    dv[q] = tread(TA(t), lrow, q);
                    xv[q] = tread(TB(t), lane & 3, q);
                }
                gb0l = fadd(gb0l, fadd(fadd(hsum4(dv[0]), hsum4(dv[1])), fadd(hsum4(dv[2]), hsum4(dv[3]))));
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) gW04 = mfma4x4(dv[q][e], xv[q][e], gW04);
            } else {
                const f32x4 fb = tread(TB(t), j, g);
#pragma unroll
                for (int m = 0; m < HT; ++m) {
                    const f32x4 fa = tread(TA(t), 16 * m + j, g);
                    gb0[m] = fadd(gb0[m], hsum4(fa));
#pragma unroll
                    for (int q = 0; q < 4; ++q) gW0[m] = mfma4(fa[q], fb[q], gW0[m]);
                }
            }
        }
        f32x4 xb[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) xb[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (NAF > 0) {
            // ≤ 4 features (the launcher's condition for these instances): x̄ on
            // v_mfma_f32_4x4x1_16b_f32 instead of a 16-row product with ≤ 4 live rows.
            // Block b = lane >> 2 takes samples 4(b & 3).. over the hidden rows of lane
            // group g = b >> 2 — exactly the δ0 values lane (g, j) holds — with W0ᵀ[i][h]
            // from the fragment of lane (g, i), i < 4 (at slot i + 4g: the LDS copy compacts
            // them); the four groups' partial sums are then added across lane groups.
            // Lane (g, j) ends with x̄[f][j] in register f.
#pragma unroll
            for (int kq = 0; kq < HT; ++kq) {
                const f32x4 w = impl::lds4(tw + G.off_w0t + kq * 1024 + ((lane & 3) + 4 * g) * 16);
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) xb[t] = mfma4x4(w[r], d0[t][kq][r], xb[t]);
            }
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) xb[t][r] = uni::xgroup_sum(xb[t][r]);
        } else {
#pragma unroll
            for (int kq = 0; kq < HT; ++kq) {
                const f32x4 w = impl::lds4(tw + G.off_w0t + kq * 1024 + lane * 16);
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) xb[t] = mfma4(w[r], d0[t][kq][r], xb[t]);
            }
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if (valid[t]) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (zxc(r) != 0xff) a.zbar[s[t] * d + zxc(r)] = zxp[t][r] + xb[t][r];
            }
            if (!sph && rnvp && g == 0 && valid[t]) {  // ū_af = z̄_af·exp(-s)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (afc(k) != 0xff) a.zbar[s[t] * d + afc(k)] = zb[t][k] * ee[t][k];
            }
        }
        lds_order();
    }

    // ---- workgroup reduction (fixed wave order) → partial[blockIdx.x] ----
    __syncthreads();
    float* R = tarea;
    // The weight matrices are summed in regions of their own: in the column-major flat
    // layout the columns of a lane group share banks (16-way on dW1's read-add-writes,
    // 4-way on the M4 blocks).  dW0, dW_out: odd column strides (h | 1, n_out | 1); dW1:
    // row-major with rows P ≡ 4 (mod 8) floats apart, so the two row quads of a 32-lane
    // group (4g apart) land 16 banks apart and its 16 columns on the rest: conflict-free.
    // The final copy gathers them back into the flat order.
    const int hp = G.h_true | 1, sp = N.n_out | 1, P1 = ((G.h_true + 3) & ~7) + 4;
    float* R0 = R + ((G.p_count + 3) & ~3);
    float* R1 = R0 + ((hp * G.n_in + 3) & ~3);
    float* R2 = R1 + ((NH == 1 ? G.h_true * P1 : 0) + 3 & ~3);
    const int rn = (int)(R2 - R) + sp * G.h_true;
    for (int i = tid; i < rn; i += NT) R[i] = 0.f;
#pragma unroll
    for (int m = 0; m < HT; ++m) gb0[m] = uni::xgroup_sum(gb0[m]);
#pragma unroll
    for (int m = 0; m < NHT; ++m) gbh[m] = uni::xgroup_sum(gbh[m]);
    gbo = uni::xgroup_sum(gbo);
    __syncthreads();
    const int h = G.h_true;
    const int wo0 = G.w_off[0] - G.p_begin, bo0 = G.b_off[0] - G.p_begin;
    const int wo1 = G.w_off[1] - G.p_begin, bo1 = G.b_off[1] - G.p_begin;
    const int wo2 = G.w_off[2] - G.p_begin, bo2 = G.b_off[2] - G.p_begin;
    for (int w = 0; w < NW; ++w) {
        if (wave == w) {
            if constexpr (M4) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (i < N.n_out && lane < h) R2[i + sp * lane] += gWo4[i];
                    const int row = 4 * (lane >> 2) + i, col = lane & 3;
                    if (row < h && col < G.n_in) R0[row + hp * col] += gW04[i];
                }
                if (G.b_off[0] >= 0 && lane < h) R[bo0 + lane] += gb0l;
                if (g == 0 && G.b_off[2] >= 0 && j < N.n_out) R[bo2 + j] += gbo;
            } else {
#pragma unroll
                for (int m = 0; m < HT; ++m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = 16 * m + 4 * g + r;
                        if (row < h && j < G.n_in) R0[row + hp * j] += gW0[m][r];
                        const int ob = 16 * m + j;  // output Dense: row o = 4g + r, column ob
                        if (4 * g + r < N.n_out && ob < h) R2[(4 * g + r) + sp * ob] += gWo[m][r];
                    }
                if (g == 0) {
#pragma unroll
                    for (int m = 0; m < HT; ++m)
                        if (G.b_off[0] >= 0 && 16 * m + j < h) R[bo0 + 16 * m + j] += gb0[m];
                    if (G.b_off[2] >= 0 && j < N.n_out) R[bo2 + j] += gbo;
                }
            }
            if constexpr (NH == 1) {
#pragma unroll
                for (int ma = 0; ma < HT; ++ma)
#pragma unroll
                    for (int mb = 0; mb < HT; ++mb)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 16 * ma + 4 * g + r, col = 16 * mb + j;
                            if (row < h && col < h) R1[col + P1 * row] += gWh[ma][mb][r];
                        }
                if (g == 0) {
#pragma unroll
                    for (int m = 0; m < HT; ++m)
                        if (G.b_off[1] >= 0 && 16 * m + j < h) R[bo1 + 16 * m + j] += gbh[m];
                }
            }
        }
        __syncthreads();
    }
    float* dst = a.partial + (int64_t)blockIdx.x * a.p_total + G.p_begin;
    for (int i = tid; i < G.p_count; i += NT) {
        const int k0 = i - wo0, k1 = i - wo1, k2 = i - wo2;
        float v = R[i];
        if (k0 >= 0 && k0 < h * G.n_in) {
            const int col = k0 / h;
            v = R0[(k0 - col * h) + hp * col];
        } else if (NH == 1 && k1 >= 0 && k1 < h * h) {
            const int col = k1 / h;
            v = R1[col + P1 * (k1 - col * h)];
        } else if (k2 >= 0 && k2 < N.n_out * h) {
            const int col = k2 / N.n_out;
            v = R2[(k2 - col * N.n_out) + sp * col];
        }
        dst[i] = v;
    }
}

template <int HT, int NH, int AM, bool SPLIT = false, int NAF = 0>
void* train_kernel_ptr() {
    return reinterpret_cast<void*>(&train_net_kernel<HT, NH, AM, SPLIT, NAF>);
}

}  // namespace df
