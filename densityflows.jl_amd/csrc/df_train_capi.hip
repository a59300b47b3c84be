// df_train_capi.hip — the training entry points of the C ABI (df_train_*).
//
// Host side of one train! step (src/Flows.jl:396-414); the device work is in
// df_train.hip / df_train_impl.h, the inverse pass with per-layer outputs in
// the specialised chain kernel (df_uniform_impl.h, ChainArgs::snap).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "df_handle.h"
#include "df_ltrain.h"
#include "df_train.h"

using namespace df;
using namespace df::api;

namespace {

struct SweepOp {
    int layer;   // index in plan.layers
    int net;     // index in df_train::nets, -1 for a NormalizationLayer
    int phase;   // TR_PHASE_S / TR_PHASE_T
};

int round16(int v) { return (v + 15) / 16 * 16; }

int pow2_tiles(int rows) {
    int t = 1;
    while (16 * t < rows) t *= 2;
    return t;
}

// Layer-wise path: one packed GEMM operand (W or Wᵀ) of one Dense.
struct LOp {
    int mt = 0;              // output row tiles (power of two <= 16)
    int nkq = 0;             // k-quads of the contraction
    int chunk_kq = 1;        // k-quads per LDS chunk
    int64_t frag = 0;        // byte offset in the layer-wise blob
    int64_t bias = -1;       // float offset of the padded bias (forward only)
    int64_t sfrag = -1;      // SPLIT planes [c][m][p][lane][8] in the split blob (Wᵀ of hidden-256 Denses)
};

struct LDense {
    int in_dim = 0, out_dim = 0, act = 0;
    int w_off = 0, b_off = -1;
    LOp fwd, bwd;            // acc = W·in (out rows) ; acc = Wᵀ·δ (in rows)
};

struct LNet {
    std::vector<LDense> dn;  // Dense(in,h,σ0), hidden..., Dense(h,out,σo)
    bool pre = false;        // a hidden σ needs its pre-activation for σ' (softplus, logcosh, swish):
                             // the sweep recomputes the net and stores σ'(x) beside H
};

// every activation the plan accepts has a derivative rule (df_train_impl.h act_grad/act_dx)
bool act_trainable(int a) { return a >= DF_ACT_IDENTITY && a <= DF_ACT_SWISH; }

bool act_needs_pre(int a) { return a == DF_ACT_SOFTPLUS || a == DF_ACT_LOGCOSH || a == DF_ACT_SWISH; }

}  // namespace

// One captured train step (df_train_step_graph): valid while the buffers it
// names are the ones it was captured with.
struct TrainGraph {
    const void* x = nullptr;
    const void* theta = nullptr;
    const void* lp = nullptr;
    int64_t batch = 0, n_total = 0, cap_gen = -1, partial_gen = -1;
    int flow = -1;                    // the θ convention it was recorded with (θ normalised in-kernel or not)
    int seen = 0;                     // eager runs with this key (captured on the second)
    hipGraphExec_t exec = nullptr;
    uint64_t last_use = 0;
};

struct df_train {
    df_chain* c = nullptr;
    df_adam opt{};
    float* d_bt = nullptr;            // device βᵗ of the next update (Adam), [β1ᵗ, β2ᵗ]
    int64_t cap_gen = 0;              // bumped when the batch-sized buffers are reallocated
    hipStream_t cap_stream = nullptr; // capture stream of df_train_step_graph
    std::vector<TrainGraph> graphs;
    uint64_t use_clock = 0;
    int64_t P = 0;
    int amode = 0;                    // fused kernel activation mode (trn::AM_*)
    std::vector<GNet> nets;
    std::vector<int> net_nh;
    std::vector<SweepOp> ops;
    std::vector<uint8_t> tblob;
    std::vector<int32_t> tdst, tsrc;
    float* d_params = nullptr;
    float* d_m = nullptr;
    float* d_v = nullptr;
    float* d_grad = nullptr;
    float* d_partial = nullptr;
    void* d_tblob = nullptr;
    void* d_pdst = nullptr;
    void* d_psrc = nullptr;
    void* d_tdst = nullptr;
    void* d_tsrc = nullptr;
    float* d_snap = nullptr;
    float* d_zbar = nullptr;
    float* d_ebuf = nullptr;
    double* d_lpsum = nullptr;
    bool debug = false;               // df_train_set_debug: refuse updates on a non-finite loss
    int theta_input = DF_THETA_AUTO;  // df_train_set_theta_input
    const double* last_lp = nullptr;  // Σ logpdf written by the last df_train_gradient
    int64_t last_n = 0;               // ... and the n_total it was taken over
    int64_t cap = 0;       // batch capacity of snap / zbar / ebuf
    int grid = 0;          // workgroups of a full net launch (resident on the device)
    size_t lds_max = 0;
    // layer-wise path (hidden width > 64, deep or wide-output conditioners)
    bool layerwise = false;
    std::vector<LNet> lnets;
    std::vector<uint8_t> lblob;      // fragments (W and Wᵀ) then padded biases
    std::vector<int32_t> ldst, lsrc; // repack map (float index ← trainables index)
    std::vector<uint8_t> tsblob;     // SPLIT W1ᵀ planes of the fused path (GNet::st_src)
    std::vector<int32_t> tsdst, tssrc; // repack map (byte offset ← trainables index·4 + plane)
    void* d_tsblob = nullptr;
    void* d_tsdst = nullptr;
    void* d_tssrc = nullptr;
    std::vector<uint8_t> lsblob;     // SPLIT planes of the layer-wise Wᵀ operands (LOp::sfrag)
    std::vector<int32_t> lsdst, lssrc; // repack map (byte offset ← trainables index·4 + plane)
    void* d_lsblob = nullptr;
    void* d_lsdst = nullptr;
    void* d_lssrc = nullptr;
    void* d_lblob = nullptr;
    void* d_ldst = nullptr;
    void* d_lsrc = nullptr;
    int lgrid = 0;                   // workgroups of the dW kernels (partial rows)
    int lwidth = 16;                 // widest activation row (floats)
    int lmax_h = 1;                  // activation buffers needed (hidden Denses + 1)
    std::vector<float*> d_lh, d_ld; // H_k and δ_k buffers [cap][lwidth]
    std::vector<float*> d_lv;       // σ'(x_k) buffers [cap][lwidth] (nets with LNet::pre)
    bool any_pre = false;
    float* d_lyp[2] = {nullptr, nullptr};  // ȳ  [cap][lwidth], by net parity
    float* d_lbp[2] = {nullptr, nullptr};  // δ of the last hidden Dense [cap][lwidth], by net parity
    float* d_lx = nullptr;           // gathered conditioner input [cap][lwidth]
    // hidden activations kept by the inverse pass (generic kernel): the sweep then
    // skips the forward recompute.  [(layer·2 + net)·lmax_h + k][B][lwidth]
    float* d_hsave = nullptr;
    bool hsave_on = false;
    // H0-free sweep (round 5; wide SPLIT chains of relu hidden-256 nets, DF_SWEEP_H0FREE): the
    // inverse pass keeps each net's features vcat(θ, u)[axis_nn] ([layer·2 + net][B][32])
    // and H1 only (d_hsave with one slot per net); the split dW1 recomputes H0 from the
    // features and writes its relu mask (d_hmask, 1 KiB per 32 samples) for the W1ᵀδ1 epilogue
    bool fmode = false;
    int sweep_req = DF_SWEEP_AUTO;   // df_train_create_ex: the requested form (df_sweep_form)
    bool separate = false;           // DF_SWEEP_SEPARATE: unmerged dW / front launches
    float* d_fsave = nullptr;
    uint32_t* d_hmask = nullptr;
    // repack maps of the chain's wide-kernel blob and biases (plan.wide)
    void* d_wdst = nullptr;
    void* d_wsrc = nullptr;
    void* d_wbdst = nullptr;
    void* d_wbsrc = nullptr;
    // repack maps of the chain's SPLIT blobs (plan.split, plan.wsplit)
    void* d_sdst = nullptr;
    void* d_ssrc = nullptr;
    void* d_wsdst = nullptr;
    void* d_wssrc = nullptr;
};

namespace {

void drop_graphs(df_train* t) {
    for (TrainGraph& g : t->graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    t->graphs.clear();
}

void free_all(df_train* t) {
    drop_graphs(t);
    if (t->cap_stream) (void)hipStreamDestroy(t->cap_stream);
    t->cap_stream = nullptr;
    if (t->d_bt) (void)hipFree(t->d_bt);
    t->d_bt = nullptr;
    void* ptrs[] = {t->d_params, t->d_m,    t->d_v,    t->d_grad, t->d_partial, t->d_tblob, t->d_pdst,
                    t->d_psrc,   t->d_tdst, t->d_tsrc, t->d_snap, t->d_zbar,    t->d_ebuf,  t->d_lpsum,
                    t->d_lblob,  t->d_ldst, t->d_lsrc, t->d_lyp[0], t->d_lyp[1], t->d_lbp[0], t->d_lbp[1], t->d_lx, t->d_hsave,
                    t->d_wdst,   t->d_wsrc, t->d_wbdst, t->d_wbsrc, t->d_sdst, t->d_ssrc,
                    t->d_wsdst, t->d_wssrc, t->d_lsblob, t->d_lsdst, t->d_lssrc,
                    t->d_tsblob, t->d_tsdst, t->d_tssrc, t->d_fsave, t->d_hmask};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (float* p : t->d_lh)
        if (p) (void)hipFree(p);
    for (float* p : t->d_ld)
        if (p) (void)hipFree(p);
    for (float* p : t->d_lv)
        if (p) (void)hipFree(p);
}

// Pack A = W (transposed = false: rows = out, k = in) or Wᵀ (rows = in, k = out)
// as fragments [kq][m][lane][4]: A[16m + (lane&15)][16kq + 4(lane>>4) + r].
LOp pack_lop(df_train* t, const Plan& P, const LDense& D, bool transposed) {
    LOp op;
    const int rows = transposed ? D.in_dim : D.out_dim;
    const int kdim = transposed ? D.out_dim : D.in_dim;
    op.mt = pow2_tiles(rows);
    op.nkq = (kdim + 15) / 16;
    op.chunk_kq = std::max(1, kLChunkBytes / (op.mt * 1024));
    op.frag = (int64_t)t->lblob.size();
    const size_t bytes = (size_t)op.nkq * op.mt * 1024;
    t->lblob.resize(t->lblob.size() + bytes, 0);
    float* f = reinterpret_cast<float*>(t->lblob.data() + op.frag);
    const int64_t f0 = op.frag / 4;
    for (int kq = 0; kq < op.nkq; ++kq)
        for (int m = 0; m < op.mt; ++m)
            for (int lane = 0; lane < 64; ++lane)
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * m + (lane & 15), k = 16 * kq + 4 * (lane >> 4) + r;
                    if (i >= rows || k >= kdim) continue;
                    const int orow = transposed ? k : i, icol = transposed ? i : k;  // W[orow, icol]
                    const int64_t src = D.w_off + orow + (int64_t)D.out_dim * icol;
                    const int64_t q = (((int64_t)kq * op.mt + m) * 64 + lane) * 4 + r;
                    f[q] = P.trainables[src];
                    t->ldst.push_back((int32_t)(f0 + q));
                    t->lsrc.push_back((int32_t)src);
                }
    // SPLIT planes of a hidden-256 Wᵀ (the ldense_kernel SPLIT instances), and of a first
    // Dense's W0ᵀ over a 256-wide hidden layer (≤ 64 conditioner inputs: the x̄ product
    // of the SPLIT W1ᵀδ1 epilogue)
    if (transposed && (op.mt == 16 || (op.mt <= 4 && op.nkq == 16)) && op.nkq % 2 == 0 && !t->c->exact) {
        op.sfrag = (int64_t)t->lsblob.size();
        t->lsblob.resize(t->lsblob.size() + (size_t)(op.nkq / 2) * op.mt * 3072, 0);
        for (int c = 0; c < op.nkq / 2; ++c)
            for (int m = 0; m < op.mt; ++m)
                for (int p = 0; p < 3; ++p)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int e = 0; e < 8; ++e) {
                            const int i = 16 * m + (lane & 15), g = lane >> 4;
                            const int k = 32 * c + 16 * (e >> 2) + 4 * g + (e & 3);
                            if (i >= rows || k >= kdim) continue;
                            const int64_t src = D.w_off + k + (int64_t)D.out_dim * i;  // Wᵀ[i, k] = W[k, i]
                            const int64_t at = op.sfrag + ((((int64_t)c * op.mt + m) * 3 + p) * 64 + lane) * 16 + 2 * e;
                            const uint16_t h = bf16_split_plane(P.trainables[src], p);
                            std::memcpy(&t->lsblob[at], &h, 2);
                            t->lsdst.push_back((int32_t)at);
                            t->lssrc.push_back((int32_t)(src * 4 + p));
                        }
    }
    return op;
}

void pack_lbias(df_train* t, const Plan& P, const LDense& D, LOp& op) {
    if (D.b_off < 0) return;
    op.bias = (int64_t)t->lblob.size() / 4;
    t->lblob.resize(t->lblob.size() + (size_t)op.mt * 64, 0);
    float* f = reinterpret_cast<float*>(t->lblob.data()) + op.bias;
    for (int r = 0; r < D.out_dim; ++r) {
        f[r] = P.trainables[D.b_off + r];
        t->ldst.push_back((int32_t)(op.bias + r));
        t->lsrc.push_back(D.b_off + r);
    }
}

int build_lnets(df_train* t) {
    const Plan& P = t->c->plan;
    t->ops.clear();
    t->lnets.clear();
    for (int li = 0; li < P.n_layers; ++li) {
        const DevLayer& L = P.layers[li];
        if (L.kind == DF_LAYER_NORM) {
            t->ops.push_back({li, -1, TR_PHASE_T});
            continue;
        }
        auto add = [&](int d0, int nd, int phase) -> int {
            LNet net;
            for (int k = 0; k < nd; ++k) {
                const DevDense& DD = P.denses[d0 + k];
                if (!act_trainable(DD.act))
                    return set_err(DF_ERR_UNSUPPORTED, "unknown activation");
                LDense D;
                D.in_dim = DD.in_dim;
                D.out_dim = DD.n_out;
                D.act = DD.act;
                D.w_off = DD.w_off;
                D.b_off = DD.b_off;
                D.fwd = pack_lop(t, P, D, false);
                pack_lbias(t, P, D, D.fwd);
                D.bwd = pack_lop(t, P, D, true);
                t->lwidth = std::max({t->lwidth, 16 * D.fwd.mt, 16 * D.bwd.mt});
                if (k + 1 < nd && act_needs_pre(D.act)) net.pre = true;
                net.dn.push_back(D);
            }
            t->lmax_h = std::max(t->lmax_h, nd - 1);
            t->any_pre = t->any_pre || net.pre;
            t->lnets.push_back(net);
            t->ops.push_back({li, (int)t->lnets.size() - 1, phase});
            return DF_OK;
        };
        int rc = DF_OK;
        if (L.kind == DF_LAYER_RNVP) rc = add(L.s_dense0, L.s_ndense, TR_PHASE_S);
        if (rc == DF_OK) rc = add(L.t_dense0, L.t_ndense, TR_PHASE_T);
        if (rc != DF_OK) return rc;
    }
    t->lblob.resize(t->lblob.size() + 16, 0);
    return DF_OK;
}

// Transposed fragments of one net (W0ᵀ, W_hᵀ) appended to t->tblob with
// their trainables index map.
void pack_transposed(df_train* t, const Plan& P, GNet& g, const DevDense& D0, const DevDense* D1, int ht) {
    const int h = g.h_true;
    const size_t base = t->tblob.size();
    g.t_src = (int64_t)base;
    g.off_w0t = 0;
    g.off_ht = ht * 1024;
    const int bytes = ht * 1024 + (D1 ? ht * ht * 1024 : 0);
    g.t_bytes = bytes;
    t->tblob.resize(base + bytes, 0);
    float* f = reinterpret_cast<float*>(t->tblob.data() + base);
    const int64_t f0 = (int64_t)base / 4;
    auto put = [&](int64_t q, int64_t src) {
        f[q] = P.trainables[src];
        t->tdst.push_back((int32_t)(f0 + q));
        t->tsrc.push_back((int32_t)src);
    };
    // W0ᵀ: [kq][lane (i,g)][r] = W0[16kq + 4g + r, i]
    for (int kq = 0; kq < ht; ++kq)
        for (int lane = 0; lane < 64; ++lane)
            for (int r = 0; r < 4; ++r) {
                const int i = lane & 15, a = 16 * kq + 4 * (lane >> 4) + r;
                if (a < h && i < g.n_in) put((int64_t)(kq * 64 + lane) * 4 + r, D0.w_off + a + (int64_t)h * i);
            }
    if (D1) {  // W1ᵀ: [kq][m][lane (i,g)][r] = W1[16kq + 4g + r, 16m + i]
        const int64_t o = g.off_ht / 4;
        for (int kq = 0; kq < ht; ++kq)
            for (int m = 0; m < ht; ++m)
                for (int lane = 0; lane < 64; ++lane)
                    for (int r = 0; r < 4; ++r) {
                        const int a = 16 * kq + 4 * (lane >> 4) + r, b = 16 * m + (lane & 15);
                        if (a < h && b < h)
                            put(o + ((int64_t)(kq * ht + m) * 64 + lane) * 4 + r, D1->w_off + a + (int64_t)h * b);
                    }
    }
}

int build_nets(df_train* t) {
    const Plan& P = t->c->plan;
    if (!P.uniform || !P.outv)
        return set_err(DF_ERR_UNSUPPORTED,
                       "training needs every conditioner in the default _dflt_net shape (hidden width <= 64) "
                       "with <= 4 transformed dims per layer");
    const int ht = P.ht;
    for (int li = 0; li < P.n_layers; ++li) {
        const DevLayer& L = P.layers[li];
        if (L.kind == DF_LAYER_NORM) {
            t->ops.push_back({li, -1, TR_PHASE_T});
            continue;
        }
        const ULayer& U = P.ulayers[li];
        auto add = [&](const UNet& u0, int d0, int nd, int phase) -> int {
            if (u0.nh > 1) return set_err(DF_ERR_UNSUPPORTED, "training supports n_sublayers <= 2 (one hidden Dense)");
            const DevDense& D0 = P.denses[d0];
            const DevDense* D1 = u0.nh == 1 ? &P.denses[d0 + 1] : nullptr;
            const DevDense& DO = P.denses[d0 + nd - 1];
            for (int k = 0; k < nd; ++k)
                if (!act_trainable(P.denses[d0 + k].act))
                    return set_err(DF_ERR_UNSUPPORTED, "unknown activation");
            GNet g{};
            g.u = u0;
            g.n_in = D0.in_dim;
            g.h_true = D0.n_out;
            // the net's bytes inside its stage: [off_w0, end of the output GEMV block)
            int lo = u0.off_w0;
            lo = std::min(lo, u0.off_b0);
            if (u0.nh) lo = std::min(lo, u0.off_h);
            lo = std::min(lo, u0.off_out);
            const int hi = u0.off_out + round16((u0.n_out * 16 * ht + 4) * 4);
            g.fwd_src = P.stages[u0.stage].src_off + lo;
            g.fwd_bytes = round16(hi - lo);
            g.u.off_w0 -= lo;
            g.u.off_b0 -= lo;
            if (u0.nh) g.u.off_h -= lo;
            g.u.off_out -= lo;
            g.w_off[0] = D0.w_off;
            g.b_off[0] = D0.b_off;
            g.w_off[1] = D1 ? D1->w_off : D0.w_off;
            g.b_off[1] = D1 ? D1->b_off : -1;
            g.w_off[2] = DO.w_off;
            g.b_off[2] = DO.b_off;
            g.p_begin = D0.w_off;
            int end = 0;
            for (int k = 0; k < nd; ++k) {
                const DevDense& D = P.denses[d0 + k];
                end = std::max(end, D.w_off + D.in_dim * D.n_out);
                if (D.b_off >= 0) end = std::max(end, D.b_off + D.n_out);
            }
            g.p_count = end - g.p_begin;
            pack_transposed(t, P, g, D0, D1, ht);
            // SPLIT: the net's region of the chain's SPLIT blob and its W1ᵀ planes
            if (use_split(t->c) && D1 && t->amode == trn::AM_RELU && (ht == 2 || ht == 4)) {
                const ULayer& SU = P.sulayers[li];
                const UNet& s0 = (phase == TR_PHASE_S) ? SU.s : SU.t;
                const int slo = s0.off_w0;
                const int shi = s0.off_out + round16((s0.n_out * 16 * ht + 4) * 4);
                g.split = 1;
                g.su = s0;
                g.su.off_w0 -= slo;
                g.su.off_h -= slo;
                g.su.off_out -= slo;
                g.sfwd_src = P.sstages[s0.stage].src_off + slo;
                g.sfwd_bytes = round16(shi - slo);
                g.st_src = (int64_t)t->tsblob.size();
                g.st_bytes = (ht / 2) * ht * 3072;
                t->tsblob.resize(t->tsblob.size() + g.st_bytes, 0);
                const int h = g.h_true;
                for (int c = 0; c < ht / 2; ++c)
                    for (int m = 0; m < ht; ++m)
                        for (int p = 0; p < 3; ++p)
                            for (int lane = 0; lane < 64; ++lane)
                                for (int e = 0; e < 8; ++e) {
                                    const int i = 16 * m + (lane & 15), gg = lane >> 4;
                                    const int k = 32 * c + 16 * (e >> 2) + 4 * gg + (e & 3);
                                    if (i >= h || k >= h) continue;
                                    const int64_t src = D1->w_off + k + (int64_t)h * i;  // W1ᵀ[i, k] = W1[k, i]
                                    const int64_t at =
                                        g.st_src + ((((int64_t)c * ht + m) * 3 + p) * 64 + lane) * 16 + 2 * e;
                                    const uint16_t hv = bf16_split_plane(P.trainables[src], p);
                                    std::memcpy(&t->tsblob[at], &hv, 2);
                                    t->tsdst.push_back((int32_t)at);
                                    t->tssrc.push_back((int32_t)(src * 4 + p));
                                }
            }
            t->nets.push_back(g);
            t->net_nh.push_back(u0.nh);
            t->ops.push_back({li, (int)t->nets.size() - 1, phase});
            return DF_OK;
        };
        int rc = DF_OK;
        if (L.kind == DF_LAYER_RNVP) rc = add(U.s, L.s_dense0, L.s_ndense, TR_PHASE_S);
        if (rc == DF_OK) rc = add(U.t, L.t_dense0, L.t_ndense, TR_PHASE_T);
        if (rc != DF_OK) return rc;
    }
    t->tblob.resize(t->tblob.size() + 16, 0);
    return DF_OK;
}

// The H0-free sweep (df_train::fmode) applies when the inverse pass runs on the wide SPLIT
// kernel and every conditioner is its shape: Dense(≤ 32, 256, relu), Dense(256, 256, relu),
// Dense(256, ≤ 32), with the fused front and the split dW1.
bool fmode_eligible(const df_train* t) {
    const df_chain* c = t->c;
    const Plan& P = c->plan;
    if (!t->layerwise || !P.wide || c->no_wide || !use_wsplit(c) || c->exact || P.uniform) return false;
    if (t->sweep_req != DF_SWEEP_AUTO && t->sweep_req != DF_SWEEP_H0FREE && t->sweep_req != DF_SWEEP_LAYERWISE)
        return false;
    for (const LNet& N : t->lnets) {
        if (N.pre || N.dn.size() != 3) return false;
        const LDense &D0 = N.dn[0], &D1 = N.dn[1], &D2 = N.dn[2];
        if (D0.act != DF_ACT_RELU || D1.act != DF_ACT_RELU) return false;
        if (D0.in_dim > 32 || D0.out_dim != 256 || D1.in_dim != 256 || D1.out_dim != 256) return false;
        // (the feature rows the split dW0 / H0 recompute read are 32 floats: 16 · bwd.mt <= 32)
        if (D2.fwd.mt > 2 || D0.bwd.mt > 2 || D1.bwd.sfrag < 0) return false;
    }
    return true;
}

int ensure_capacity(df_train* t, int64_t batch) {
    if (batch <= t->cap) return DF_OK;
    t->cap_gen++;  // captured train steps name the old buffers
    const Plan& P = t->c->plan;
    for (float** p : {&t->d_snap, &t->d_zbar, &t->d_ebuf})
        if (*p) {
            (void)hipFree(*p);
            *p = nullptr;
        }
    t->cap = 0;
    const int64_t cap = std::max<int64_t>(batch, 1024);
    for (float** p : {&t->d_lyp[0], &t->d_lyp[1], &t->d_lbp[0], &t->d_lbp[1], &t->d_lx, &t->d_hsave, &t->d_fsave})
        if (*p) {
            (void)hipFree(*p);
            *p = nullptr;
        }
    if (t->d_hmask) (void)hipFree(t->d_hmask);
    t->d_hmask = nullptr;
    for (auto* v : {&t->d_lh, &t->d_ld, &t->d_lv}) {
        for (float* p : *v)
            if (p) (void)hipFree(p);
        v->clear();
    }
    const int ew = t->layerwise ? 32 : 4;  // exp(-s) row width
    if (hipMalloc(reinterpret_cast<void**>(&t->d_snap), sizeof(float) * P.n_layers * cap * P.d) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_zbar), sizeof(float) * cap * P.d) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_ebuf), sizeof(float) * cap * ew) != hipSuccess)
        return set_err(DF_ERR_NOMEM, "hipMalloc failed (training activations)");
    if (t->layerwise) {
        const size_t row = sizeof(float) * (size_t)cap * t->lwidth;
        if (hipMalloc(reinterpret_cast<void**>(&t->d_lyp[0]), row) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&t->d_lyp[1]), row) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&t->d_lbp[0]), row) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&t->d_lbp[1]), row) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&t->d_lx), row) != hipSuccess)
            return set_err(DF_ERR_NOMEM, "hipMalloc failed (training activations)");
        // keep the inverse pass's hidden activations when the chain runs on the generic
        // kernel and they fit (else the sweep recomputes them)
        t->hsave_on = false;
        if (!P.uniform && t->sweep_req != DF_SWEEP_RECOMPUTE) {
            // fmode: H1 only, plus the 32-float feature rows and the relu-mask buffer; else
            // H0 and H1 of every net.  Whatever does not fit falls back: fmode → kept H0/H1
            // → recompute (the sweep's forms, struct df_train)
            size_t free_b = 0, total_b = 0;
            const bool info = hipMemGetInfo(&free_b, &total_b) == hipSuccess;
            auto try_keep = [&](bool fm) {
                const size_t hbytes = row * (size_t)P.n_layers * 2 * (fm ? 1 : t->lmax_h);
                const size_t fbytes = fm ? sizeof(float) * (size_t)cap * 32 * P.n_layers * 2 : 0;
                const size_t mbytes = fm ? (size_t)(cap + 31) / 32 * 1024 : 0;
                if (!info || hbytes + fbytes + mbytes >= free_b / 2) return false;
                if (hipMalloc(reinterpret_cast<void**>(&t->d_hsave), hbytes) == hipSuccess &&
                    (!fm || (hipMalloc(reinterpret_cast<void**>(&t->d_fsave), fbytes) == hipSuccess &&
                             hipMalloc(reinterpret_cast<void**>(&t->d_hmask), mbytes) == hipSuccess)))
                    return true;
                for (float** p : {&t->d_hsave, &t->d_fsave})
                    if (*p) {
                        (void)hipFree(*p);
                        *p = nullptr;
                    }
                if (t->d_hmask) (void)hipFree(t->d_hmask);
                t->d_hmask = nullptr;
                return false;
            };
            if (t->fmode && !try_keep(true)) t->fmode = false;  // sized for H0 and H1 below
            if (t->fmode || try_keep(false)) t->hsave_on = true;
            (void)hipGetLastError();
        }
        for (int k = 0; k <= t->lmax_h; ++k) {
            float *h = nullptr, *dl = nullptr;
            if (hipMalloc(reinterpret_cast<void**>(&h), row) != hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&dl), row) != hipSuccess) {
                if (h) (void)hipFree(h);
                return set_err(DF_ERR_NOMEM, "hipMalloc failed (training activations)");
            }
            t->d_lh.push_back(h);
            t->d_ld.push_back(dl);
            if (t->any_pre && k < t->lmax_h) {
                float* dv = nullptr;
                if (hipMalloc(reinterpret_cast<void**>(&dv), row) != hipSuccess)
                    return set_err(DF_ERR_NOMEM, "hipMalloc failed (training activations)");
                t->d_lv.push_back(dv);
            }
        }
    }
    t->cap = cap;
    return DF_OK;
}

int repack(df_train* t, hipStream_t st) {
    df_chain* c = t->c;
    const Plan& P = c->plan;
    hipError_t e = launch_repack(static_cast<float*>(c->d_blob), static_cast<const int32_t*>(t->d_pdst),
                                 static_cast<const int32_t*>(t->d_psrc), (int64_t)P.pack_dst.size(), t->d_params, st);
    if (e == hipSuccess && !t->tdst.empty())
        e = launch_repack(static_cast<float*>(t->d_tblob), static_cast<const int32_t*>(t->d_tdst),
                          static_cast<const int32_t*>(t->d_tsrc), (int64_t)t->tdst.size(), t->d_params, st);
    if (e == hipSuccess && P.wide) {
        e = launch_repack(static_cast<float*>(c->d_wblob), static_cast<const int32_t*>(t->d_wdst),
                          static_cast<const int32_t*>(t->d_wsrc), (int64_t)P.wpack_dst.size(), t->d_params, st);
        if (e == hipSuccess)
            e = launch_repack(static_cast<float*>(c->d_wbias), static_cast<const int32_t*>(t->d_wbdst),
                              static_cast<const int32_t*>(t->d_wbsrc), (int64_t)P.wbias_dst.size(), t->d_params, st);
    }
    if (e == hipSuccess && P.split)
        e = launch_repack_split(static_cast<uint8_t*>(c->d_sblob), static_cast<const int32_t*>(t->d_sdst),
                                static_cast<const int32_t*>(t->d_ssrc), (int64_t)P.spack_dst.size(), t->d_params, st);
    if (e == hipSuccess && P.wsplit)
        e = launch_repack_split(static_cast<uint8_t*>(c->d_wsblob), static_cast<const int32_t*>(t->d_wsdst),
                                static_cast<const int32_t*>(t->d_wssrc), (int64_t)P.wspack_dst.size(), t->d_params,
                                st);
    if (e == hipSuccess && !t->ldst.empty())
        e = launch_repack(static_cast<float*>(t->d_lblob), static_cast<const int32_t*>(t->d_ldst),
                          static_cast<const int32_t*>(t->d_lsrc), (int64_t)t->ldst.size(), t->d_params, st);
    if (e == hipSuccess && !t->tsdst.empty())
        e = launch_repack_split(static_cast<uint8_t*>(t->d_tsblob), static_cast<const int32_t*>(t->d_tsdst),
                                static_cast<const int32_t*>(t->d_tssrc), (int64_t)t->tsdst.size(), t->d_params, st);
    if (e == hipSuccess && !t->lsdst.empty())
        e = launch_repack_split(static_cast<uint8_t*>(t->d_lsblob), static_cast<const int32_t*>(t->d_lsdst),
                                static_cast<const int32_t*>(t->d_lssrc), (int64_t)t->lsdst.size(), t->d_params, st);
    return e == hipSuccess ? DF_OK : hip_err(e, "repack kernel launch");
}

// Reverse sweep of the layer-wise path (chain order; see df_ltrain.h).
int lsweep(df_train* t, const float* x, const float* theta, int64_t batch, float inv_n, bool flow, hipStream_t st) {
    df_chain* c = t->c;
    const Plan& P = c->plan;
    const int64_t bd = batch * P.d;
    const int64_t ntiles = (batch + 15) / 16;
    const unsigned dgrid =
        (unsigned)std::max<int64_t>(1, std::min<int64_t>(c->n_cu, (ntiles + kWavesPerBlock * kLTiles - 1) /
                                                                          (kWavesPerBlock * kLTiles)));
    const int W = t->lwidth;
    const uint8_t* lb = static_cast<const uint8_t*>(t->d_lblob);
    const float* lbf = static_cast<const float*>(t->d_lblob);
    const uint8_t* lsb = static_cast<const uint8_t*>(t->d_lsblob);
    const bool lsplit = !c->exact;   // the chain's arithmetic, fixed at df_chain_create
    auto sfrag_of = [&](const LOp& op, int in_kind, int epi) -> const uint8_t* {
        return (lsplit && op.sfrag >= 0 && ldense_split_supported(op.mt, in_kind, epi)) ? lsb + op.sfrag : nullptr;
    };
    hipError_t e = hipSuccess;
    auto dense = [&](const LOp& op, int in_kind, int epi, LDenseArgs a) {
        a.wfrag = lb + op.frag;
        a.bias = (op.bias >= 0 && (epi == LEPI_ACT || epi == LEPI_COUPLE)) ? lbf + op.bias : nullptr;
        a.nkq = op.nkq;
        a.chunk_kq = op.chunk_kq;
        a.sfrag = sfrag_of(op, in_kind, epi);
        const int nchunks = (op.nkq + op.chunk_kq - 1) / op.chunk_kq;
        const size_t lds = a.sfrag ? (size_t)(op.nkq / 2 > 1 ? 2 : 1) * op.mt * 3072
                                   : (size_t)(nchunks > 1 ? 2 : 1) * std::min(op.nkq, op.chunk_kq) * op.mt * 1024;
        if (e == hipSuccess) e = launch_ldense(op.mt, in_kind, epi, a, dgrid, lds, st);
    };
    // Per net op: base arguments, and whether its backward front is the fused
    // couple_bwd kernel (kept activations, <= 32 outputs, hidden <= 256).
    const size_t nops = t->ops.size();
    auto base_args = [&](const SweepOp& op) {
        const DevLayer& L = P.layers[op.layer];
        const LNet& N = t->lnets[op.net];
        LDenseArgs b{};
        b.theta = theta;
        b.tmin = flow ? c->d_bounds : nullptr;
        b.tmax = flow ? c->d_bounds + P.n : nullptr;
        b.u_in = (op.layer + 1 < P.n_layers) ? t->d_snap + (int64_t)(op.layer + 1) * bd : x;
        b.u_out = t->d_snap + (int64_t)op.layer * bd;
        b.feat = static_cast<const int32_t*>(c->d_tables) + L.feat_tab;
        b.af = static_cast<const int32_t*>(c->d_tables) + L.af_tab;
        b.n_in = N.dn[0].in_dim;
        b.zbar = t->d_zbar;
        b.ebuf = t->d_ebuf;
        b.n_af = L.n_af;
        b.phase = op.phase;
        b.kind = L.kind;
        b.inv_n = inv_n;
        b.batch = batch;
        b.d = P.d;
        b.n = P.n;
        b.ld_in = b.ld_out = b.ld_h = b.ld_x = W;
        return b;
    };
    const bool no_merge = t->separate;  // DF_SWEEP_SEPARATE
    auto keeps = [&](const SweepOp& op) { return t->hsave_on && !t->lnets[op.net].pre; };
    const bool fm = t->fmode && t->hsave_on && t->d_fsave;  // H0-free sweep (struct df_train)
    auto net_slot = [&](const SweepOp& op) { return 2 * op.layer + (op.phase == TR_PHASE_T ? 1 : 0); };
    // fmode: the net's feature rows [B][32] (written by the inverse pass)
    auto fbuf = [&](const SweepOp& op) { return t->d_fsave + (int64_t)net_slot(op) * batch * 32; };
    auto fused_front = [&](const SweepOp& op) {
        const LNet& N = t->lnets[op.net];
        const int nd = (int)N.dn.size();
        return nd >= 2 && keeps(op) && N.dn[nd - 1].fwd.mt <= 2 && N.dn[0].bwd.mt <= 4;
    };
    // H_k of a net: kept by the inverse pass, or recomputed into the shared buffers
    auto Hbuf = [&](const SweepOp& op, int k) -> float* {
        if (fm) return k == 1 ? t->d_hsave + (int64_t)net_slot(op) * batch * W : nullptr;  // H1 only
        return keeps(op) ? t->d_hsave + ((int64_t)net_slot(op) * t->lmax_h + k) * batch * W : t->d_lh[k];
    };
    // ȳ and the δ of the last hidden Dense alternate between two buffers from net to
    // net: a merged launch writes net i+1's while net i's dW products read net i's
    auto ybuf = [&](int par) { return t->d_lyp[par]; };
    auto dbuf = [&](const SweepOp& op, int k, int par) -> float* {
        return k == (int)t->lnets[op.net].dn.size() - 2 ? t->d_lbp[par] : t->d_ld[k];
    };
    // couple_bwd: output Dense + pullback → ȳ, then δ_last = (W_outᵀ ȳ) ⊙ σ'(H)
    auto front_args = [&](const SweepOp& op, int par, LDenseArgs& a, int* ht, int* mto, size_t* lds) {
        const LNet& N = t->lnets[op.net];
        const int nd = (int)N.dn.size();
        const LDense& DO = N.dn[nd - 1];
        a = base_args(op);
        a.act = DO.act;
        a.in = Hbuf(op, nd - 2);
        a.wfrag = lb + DO.fwd.frag;
        a.bias = DO.fwd.bias >= 0 ? lbf + DO.fwd.bias : nullptr;
        a.nkq = DO.fwd.nkq;
        a.w2frag = lb + DO.bwd.frag;
        a.nkq2 = DO.bwd.nkq;
        a.out = ybuf(par);
        a.out2 = dbuf(op, nd - 2, par);
        a.dact = N.dn[nd - 2].act;
        *ht = DO.bwd.mt;
        *mto = DO.fwd.mt;
        *lds = (size_t)2 * DO.bwd.mt * DO.fwd.mt * 1024;
        if (front_dwo(DO.fwd.mt)) {  // the output Dense's dW / db come from the front (partial rows: lgrid)
            a.dwo_partial = t->d_partial;
            a.dwo_p_total = t->P;
            a.dwo_w_off = DO.w_off;
            a.dwo_b_off = DO.b_off;
            a.dwo_m_true = DO.out_dim;
            a.dwo_n_true = DO.in_dim;
            *lds += front_dwo_lds(DO.bwd.mt);
        }
    };
    // dW = δ · inᵀ, db = Σ δ of every Dense of a net (per-workgroup partials)
    auto dw_args = [&](const SweepOp& op, int par, std::vector<LdwArgs>& out) -> int {
        const LNet& N = t->lnets[op.net];
        const int nd = (int)N.dn.size();
        for (int k = 0; k < nd; ++k) {
            const LDense& D = N.dn[k];
            if (k + 1 == nd && fused_front(op) && front_dwo(D.fwd.mt)) continue;  // (the front's)
            LdwArgs w{};
            w.da = (k + 1 == nd) ? ybuf(par) : dbuf(op, k, par);
            w.lda = W;
            w.m_true = D.out_dim;
            w.mta = D.fwd.mt;
            w.xb = (k == 0) ? (fm ? fbuf(op) : t->d_lx) : Hbuf(op, k - 1);
            w.ldb = (k == 0 && fm) ? 32 : W;
            w.n_true = D.in_dim;
            w.ntb = D.bwd.mt;
            w.partial = t->d_partial;
            w.p_total = t->P;
            w.w_off = D.w_off;
            w.b_off = D.b_off;
            w.batch = batch;
            if (!ldw_shape(w.mta, w.ntb, &w.wm, &w.bm, &w.bn)) return set_err(DF_ERR_UNSUPPORTED, "dW tiling");
            // hidden-256 × hidden-256 dW on bf16x3 split products (ldw_split_body)
            w.split = (lsplit && w.mta == 16 && w.ntb == 16 && w.bm == kLdwBM && w.bn == kLdwBN) ? 1 : 0;
            if (fm && k == 1) {  // dW1 with H0 recomputed from the features (and its relu mask)
                if (!w.split || nd != 3) return set_err(DF_ERR_INVALID, "internal: H0-free sweep without the split dW1");
                const WLayer& WL = P.wslayers[op.layer];
                const WNet& WN = op.phase == TR_PHASE_T ? WL.t : WL.s;
                const DevStage& S0 = P.wsstages[WN.stage0];
                w.xb = nullptr;
                w.feat = fbuf(op);
                w.w0s = static_cast<const uint8_t*>(c->d_wsblob) + S0.src_off;
                w.b0 = static_cast<const float*>(c->d_wbias) + WN.b0;
                w.hmask = t->d_hmask;
            }
            out.push_back(w);
        }
        return DF_OK;
    };

    int par = 0;               // buffer parity of the current net
    bool front_done = false;   // this net's couple_bwd ran in the previous merged launch
    for (size_t oi = 0; oi < nops; ++oi) {
        const SweepOp& op = t->ops[oi];
        const DevLayer& L = P.layers[op.layer];
        if (op.net < 0) {
            const float* xmn = static_cast<const float*>(c->d_params) + L.norm_off;
            e = launch_norm_adjoint(t->d_zbar, xmn, xmn + P.d, L.alpha, L.beta, P.d, batch, st);
            if (e != hipSuccess) return hip_err(e, "norm adjoint launch");
            front_done = false;
            continue;
        }
        const LNet& N = t->lnets[op.net];
        const int nd = (int)N.dn.size();
        const LDenseArgs b = base_args(op);
        const bool keep = keeps(op);
        const bool fused = fused_front(op);
        if (fm && !fused) return set_err(DF_ERR_INVALID, "internal: H0-free sweep without the fused front");
        // σ' argument of Dense k's output: H_k, or the stored σ'(x_k)
        auto DACT = [&](int k, LDenseArgs& a) {
            a.hprev = N.pre ? t->d_lv[k] : Hbuf(op, k);
            a.dact = N.pre ? trn::kDactStored : N.dn[k].act;
        };
        // forward (recompute): H_k = σ(W_k · in + b_k), then the output Dense + coupling pullback → ȳ
        for (int k = 0; k < nd - (fused ? 1 : 0); ++k) {
            LDenseArgs a = b;
            a.act = N.dn[k].act;
            if (k + 1 < nd && keep) {
                if (k == 0 && !fm) {  // (fmode: the inverse pass kept the features)
                    a.xsave = t->d_lx;
                    e = e == hipSuccess ? launch_gather_features(a, 16 * N.dn[0].bwd.mt, st) : e;
                }
                continue;
            }
            if (k == 0) {
                a.xsave = t->d_lx;
                if (nd == 1) {  // a single-Dense conditioner: its input is the gathered features
                    e = e == hipSuccess ? launch_gather_features(a, 16 * N.dn[0].bwd.mt, st) : e;
                    a.in = t->d_lx;
                }
            } else {
                a.in = Hbuf(op, k - 1);
            }
            if (k + 1 < nd) {
                a.out = Hbuf(op, k);
                a.dsave = N.pre ? t->d_lv[k] : nullptr;
                dense(N.dn[k].fwd, k == 0 ? LIN_GATHER : LIN_BUF, LEPI_ACT, a);
            } else {
                a.out = ybuf(par);
                dense(N.dn[k].fwd, LIN_BUF, LEPI_COUPLE, a);
            }
        }
        // dW products of this net (launched after the backward; fmode: the split dW1 first,
        // it writes the H0 relu mask the W1ᵀδ1 epilogue reads)
        std::vector<LdwArgs> jobs;
        {
            const int rc0 = dw_args(op, par, jobs);
            if (rc0 != DF_OK) return rc0;
        }
        // backward: δ_{k-1} = (W_kᵀ δ_k) ⊙ σ'(H_{k-1}); x̄ = W0ᵀ δ_0 → z̄ (identity dims)
        const float* gcur = ybuf(par);
        if (fused) {
            // output Dense + pullback + (W_outᵀ ȳ) ⊙ σ'(H) in one pass (unless the previous
            // merged launch ran it); the last W_kᵀ product carries x̄ = W0ᵀ δ0 in its epilogue
            if (!front_done) {
                LDenseArgs a;
                int ht = 0, mto = 0;
                size_t lds = 0;
                front_args(op, par, a, &ht, &mto, &lds);
                // (a front that writes dW partial rows runs on every row's workgroup)
                const unsigned fgrid = front_dwo(mto) ? (unsigned)t->lgrid : dgrid;
                if (e == hipSuccess) e = launch_couple_bwd(ht, mto, a, fgrid, lds, st);
            }
            gcur = dbuf(op, nd - 2, par);
            if (fm) {
                for (auto it = jobs.begin(); it != jobs.end(); ++it)
                    if (it->feat) {
                        if (e == hipSuccess) e = launch_ldw(*it, (unsigned)t->lgrid, st);
                        jobs.erase(it);
                        break;
                    }
            }
            bool xbar_apart = false;  // x̄ = W0ᵀδ0 as its own product (a wide first Dense)
            for (int k = nd - 2; k >= 1; --k) {
                LDenseArgs c2 = b;
                c2.in = gcur;
                DACT(k - 1, c2);
                if (fm && k == 1) {  // σ'(H0) from the mask the split dW1 just wrote
                    c2.hprev = nullptr;
                    c2.hmask = t->d_hmask;
                }
                c2.out = dbuf(op, k - 1, par);
                if (k == 1) {
                    c2.w0t = lb + N.dn[0].bwd.frag;
                    c2.w0t_mt = N.dn[0].bwd.mt;
                    c2.w0t_nkq = N.dn[0].bwd.nkq;
                    const LOp& lo = N.dn[k].bwd;
                    const int nchunks = (lo.nkq + lo.chunk_kq - 1) / lo.chunk_kq;
                    const int xepi = (fm && k == 1) ? LEPI_DACT_XBAR_MASK : LEPI_DACT_XBAR;
                    c2.sfrag = sfrag_of(lo, LIN_BUF, xepi);
                    if (fm && !c2.sfrag) return set_err(DF_ERR_INVALID, "internal: H0-free sweep without the split W1ᵀδ1");
                    // x̄ on split products when the W1ᵀδ1 product is SPLIT and W0ᵀ has planes
                    c2.w0s = (c2.sfrag && N.dn[0].bwd.sfrag >= 0 && c2.w0t_nkq <= 16) ? lsb + N.dn[0].bwd.sfrag
                                                                                     : nullptr;
                    const size_t wbytes = c2.sfrag ? (size_t)(lo.nkq / 2 > 1 ? 2 : 1) * lo.mt * 3072
                                                   : (size_t)(nchunks > 1 ? 2 : 1) * std::min(lo.nkq, lo.chunk_kq) *
                                                         lo.mt * 1024;
                    auto w0_bytes = [&]() {
                        return c2.w0s ? (size_t)(c2.w0t_nkq / 2) * c2.w0t_mt * 3072
                                      : (size_t)c2.w0t_mt * c2.w0t_nkq * 1024;
                    };
                    // W0ᵀ stays resident beside the W1ᵀ chunk buffers: with more than 32
                    // conditioner inputs its split planes (or even its f32 fragments, at 64
                    // inputs) do not fit; then the f32 fragments, or x̄ = W0ᵀδ0 as its own
                    // product after the δ0 kernel
                    constexpr size_t kLdsMax = 160 * 1024;
                    if (wbytes + w0_bytes() + 64 > kLdsMax) c2.w0s = nullptr;
                    const size_t lds2 = wbytes + w0_bytes() + 64;  // + z̄ column table
                    c2.wfrag = lb + lo.frag;
                    c2.nkq = lo.nkq;
                    c2.chunk_kq = lo.chunk_kq;
                    if (lds2 <= kLdsMax) {
                        if (e == hipSuccess) e = launch_ldense(lo.mt, LIN_BUF, xepi, c2, dgrid, lds2, st);
                    } else {
                        if (fm) return set_err(DF_ERR_INVALID, "internal: H0-free sweep with a wide first Dense");
                        c2.w0t = nullptr;
                        dense(lo, LIN_BUF, LEPI_DACT, c2);
                        xbar_apart = true;
                    }
                } else {
                    dense(N.dn[k].bwd, LIN_BUF, LEPI_DACT, c2);
                }
                gcur = dbuf(op, k - 1, par);
            }
            if (nd == 2 || xbar_apart) {
                LDenseArgs c3 = b;
                c3.in = gcur;
                dense(N.dn[0].bwd, LIN_BUF, LEPI_XBAR, c3);
            }
        }
        for (int k = nd - 1; k >= 1 && !fused; --k) {
            LDenseArgs a = b;
            a.in = gcur;
            DACT(k - 1, a);
            a.out = dbuf(op, k - 1, par);
            dense(N.dn[k].bwd, LIN_BUF, LEPI_DACT, a);
            gcur = dbuf(op, k - 1, par);
        }
        if (!fused) {
            LDenseArgs a = b;
            a.in = gcur;
            dense(N.dn[0].bwd, LIN_BUF, LEPI_XBAR, a);
        }
        if (e != hipSuccess) return hip_err(e, "layer-wise dense launch");
        // dW products of this net, merged with the next net's front when that net is the
        // next op and runs the fused front (its front reads only z̄ after this net's
        // W1ᵀδ1 kernel, the kept H, and writes the other parity's ȳ / δ_last)
        front_done = false;
        // the split 256×256 dW runs as its own launch (one wave per SIMD, ldw_split_kernel)
        for (auto it = jobs.begin(); it != jobs.end();) {
            if (!it->split) {
                ++it;
                continue;
            }
            e = launch_ldw(*it, (unsigned)t->lgrid, st);
            if (e != hipSuccess) return hip_err(e, "split dW kernel launch");
            it = jobs.erase(it);
        }
        if (!no_merge && jobs.size() <= 3) {
            SweepJob j{};
            // narrow (HBM-bound) products first, the hidden×hidden one last: even
            // workgroups run them in this order, odd ones in reverse
            std::stable_sort(jobs.begin(), jobs.end(), [](const LdwArgs& p, const LdwArgs& q) {
                return ldw_staging_samples(p) > ldw_staging_samples(q);
            });
            j.nw = (int)jobs.size();
            for (int k = 0; k < j.nw; ++k) {
                j.w[k] = jobs[k];
                j.ws[k] = ldw_staging_samples(jobs[k]);
            }
            int ht = 0, mto = 1;
            size_t lds = ldw_lds_bytes();
            if (oi + 1 < nops && t->ops[oi + 1].net >= 0 && fused_front(t->ops[oi + 1])) {
                size_t flds = 0;
                int fht = 0, fmto = 0;
                LDenseArgs fa;
                front_args(t->ops[oi + 1], par ^ 1, fa, &fht, &fmto, &flds);
                if (sweep_supported(fht, fmto)) {
                    j.front = fa;
                    j.has_front = 1;
                    ht = fht;
                    mto = fmto;
                    lds = std::max(lds, flds);
                }
            }
            e = launch_sweep(ht, mto, j, (unsigned)t->lgrid, lds, st);
            if (e != hipSuccess) return hip_err(e, "merged sweep launch");
            front_done = j.has_front != 0;
        } else {
            for (const LdwArgs& w : jobs) {
                e = launch_ldw(w, (unsigned)t->lgrid, st);
                if (e != hipSuccess) return hip_err(e, "dW kernel launch");
            }
        }
        par ^= 1;
    }
    return DF_OK;
}

}  // namespace

extern "C" {

int df_train_destroy(df_train* t) {
    if (!t) return DF_OK;
    DeviceGuard gd(t->c->device);
    free_all(t);
    t->c->n_trainers--;
    delete t;
    return DF_OK;
}

int df_train_create(df_train** out, df_chain* c, const df_adam* opt) {
    return df_train_create_ex(out, c, opt, DF_SWEEP_AUTO);
}

int df_train_create_ex(df_train** out, df_chain* c, const df_adam* opt, int sweep) {
    if (!out || !c) return set_err(DF_ERR_INVALID, "null pointer");
    *out = nullptr;
    const int form = sweep & ~DF_SWEEP_SEPARATE;
    if (form < DF_SWEEP_AUTO || form > DF_SWEEP_LAYERWISE || (sweep & ~(DF_SWEEP_SEPARATE | 7)))
        return set_err(DF_ERR_INVALID, "unknown sweep form");
    if (form == DF_SWEEP_FUSED && (sweep & DF_SWEEP_SEPARATE))
        return set_err(DF_ERR_INVALID, "DF_SWEEP_SEPARATE applies to the layer-wise forms");
    df_train* t = new (std::nothrow) df_train();
    if (!t) return set_err(DF_ERR_NOMEM, "host allocation failed");
    t->c = c;
    t->sweep_req = form;
    t->separate = (sweep & DF_SWEEP_SEPARATE) != 0;
    t->opt = opt ? *opt : df_adam{1e-3f, 0.9f, 0.999f, 1e-8f};
    if (!(t->opt.eta >= 0.f) || !(t->opt.beta1 >= 0.f && t->opt.beta1 < 1.f) ||
        !(t->opt.beta2 >= 0.f && t->opt.beta2 < 1.f) || !(t->opt.epsilon >= 0.f)) {
        delete t;
        return set_err(DF_ERR_INVALID, "invalid Adam hyper-parameters");
    }
    const Plan& P = c->plan;
    t->P = (int64_t)P.trainables.size();
    t->amode = P.relu_only ? trn::AM_RELU : trn::AM_Y;
    for (const DevDense& D : P.denses)
        if (act_needs_pre(D.act) && !P.relu_only) t->amode = trn::AM_PRE;
    // fused per-net kernel when every conditioner fits its registers, else layer-wise
    int rc = (form == DF_SWEEP_AUTO || form == DF_SWEEP_FUSED) ? build_nets(t) : DF_ERR_UNSUPPORTED;
    if (rc == DF_ERR_UNSUPPORTED && form != DF_SWEEP_FUSED) {
        t->nets.clear();
        t->net_nh.clear();
        t->ops.clear();
        t->tblob.clear();
        t->tdst.clear();
        t->tsrc.clear();
        t->tsblob.clear();
        t->tsdst.clear();
        t->tssrc.clear();
        t->layerwise = true;
        rc = build_lnets(t);
    }
    if (rc != DF_OK) {
        delete t;
        return rc;
    }
    DeviceGuard gd(c->device);
    if (!gd.ok) {
        delete t;
        return set_err(DF_ERR_HIP, "hipSetDevice failed");
    }
    c->n_trainers++;
    // LDS and resident grid of the net kernels
    for (size_t i = 0; i < t->nets.size(); ++i) t->lds_max = std::max(t->lds_max, train_net_lds(P.ht, t->nets[i]));
    if (t->lds_max > 160 * 1024) {
        df_train_destroy(t);
        return set_err(DF_ERR_UNSUPPORTED, "training kernel needs more than 160 KiB of LDS");
    }
    hipError_t e = set_train_lds_limit(t->lds_max);
    if (e != hipSuccess) {
        df_train_destroy(t);
        return hip_err(e, "hipFuncSetAttribute(train)");
    }
    int occ = 1;
    for (size_t i = 0; i < t->nets.size(); ++i) {
        int b = 1;
        if (train_net_occupancy(P.ht, t->net_nh[i], t->amode, t->lds_max, &b, t->nets[i].split != 0) == hipSuccess &&
            b >= 1)
            occ = (i == 0) ? b : std::min(occ, b);
    }
    t->grid = std::max(1, c->n_cu * occ);
    if (t->layerwise) {
        e = set_ldense_lds_limit(160 * 1024);
        if (e == hipSuccess) e = set_couple_bwd_lds_limit(64 * 1024);
        if (e == hipSuccess) e = set_sweep_lds_limit(std::max<size_t>(ldw_lds_bytes(), 64 * 1024));
        if (e != hipSuccess) {
            df_train_destroy(t);
            return hip_err(e, "hipFuncSetAttribute(layer-wise training)");
        }
        t->lgrid = std::max(1, c->n_cu);
        t->grid = t->lgrid;  // partial rows
        t->fmode = fmode_eligible(t);
        // an explicit form the chain cannot take: the H0-free sweep's shape, or kept
        // activations of a chain whose inverse pass (the specialised kernel) keeps none
        if ((form == DF_SWEEP_H0FREE && !t->fmode) || (form == DF_SWEEP_KEPT && P.uniform)) {
            df_train_destroy(t);
            return set_err(DF_ERR_UNSUPPORTED, form == DF_SWEEP_H0FREE
                                                   ? "DF_SWEEP_H0FREE needs wide SPLIT nets Dense(<=32,256,relu), "
                                                     "Dense(256,256,relu), Dense(256,<=32)"
                                                   : "DF_SWEEP_KEPT needs a chain on the generic or wide kernel");
        }
    }
    const size_t pb = sizeof(float) * (size_t)std::max<int64_t>(t->P, 4);
    if (hipMalloc(reinterpret_cast<void**>(&t->d_params), pb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_m), pb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_v), pb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_grad), pb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_partial), pb * t->grid) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_lpsum), sizeof(double)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&t->d_bt), 2 * sizeof(float)) != hipSuccess) {
        df_train_destroy(t);
        return set_err(DF_ERR_NOMEM, "hipMalloc failed (training state)");
    }
    {  // Optimisers.setup: βᵗ = β for the first update
        const float bt[2] = {t->opt.beta1, t->opt.beta2};
        if (hipMemcpy(t->d_bt, bt, sizeof(bt), hipMemcpyHostToDevice) != hipSuccess) {
            df_train_destroy(t);
            return set_err(DF_ERR_HIP, "hipMemcpy(Adam state)");
        }
    }
    if ((rc = upload(t->tblob, &t->d_tblob)) != DF_OK || (rc = upload(t->lblob, &t->d_lblob)) != DF_OK ||
        (rc = upload(t->ldst, &t->d_ldst)) != DF_OK || (rc = upload(t->lsrc, &t->d_lsrc)) != DF_OK ||
        (rc = upload(P.pack_dst, &t->d_pdst)) != DF_OK || (rc = upload(P.wpack_dst, &t->d_wdst)) != DF_OK ||
        (rc = upload(P.wpack_src, &t->d_wsrc)) != DF_OK || (rc = upload(P.wbias_dst, &t->d_wbdst)) != DF_OK ||
        (rc = upload(P.wbias_src, &t->d_wbsrc)) != DF_OK ||
        (rc = upload(P.pack_src, &t->d_psrc)) != DF_OK || (rc = upload(t->tdst, &t->d_tdst)) != DF_OK ||
        (rc = upload(t->tsrc, &t->d_tsrc)) != DF_OK || (rc = upload(P.spack_dst, &t->d_sdst)) != DF_OK ||
        (rc = upload(P.spack_src, &t->d_ssrc)) != DF_OK || (rc = upload(P.wspack_dst, &t->d_wsdst)) != DF_OK ||
        (rc = upload(P.wspack_src, &t->d_wssrc)) != DF_OK || (rc = upload(t->lsblob, &t->d_lsblob)) != DF_OK ||
        (rc = upload(t->lsdst, &t->d_lsdst)) != DF_OK || (rc = upload(t->lssrc, &t->d_lssrc)) != DF_OK ||
        (rc = upload(t->tsblob, &t->d_tsblob)) != DF_OK || (rc = upload(t->tsdst, &t->d_tsdst)) != DF_OK ||
        (rc = upload(t->tssrc, &t->d_tssrc)) != DF_OK) {
        std::string m = last_error();
        df_train_destroy(t);
        return set_err(rc, m);
    }
    if (t->P > 0 && (hipMemcpy(t->d_params, P.trainables.data(), sizeof(float) * t->P, hipMemcpyHostToDevice) !=
                         hipSuccess ||
                     hipMemset(t->d_m, 0, sizeof(float) * t->P) != hipSuccess ||
                     hipMemset(t->d_v, 0, sizeof(float) * t->P) != hipSuccess ||
                     hipMemset(t->d_grad, 0, sizeof(float) * t->P) != hipSuccess)) {
        df_train_destroy(t);
        return set_err(DF_ERR_HIP, "initialising the training state failed");
    }
    *out = t;
    return DF_OK;
}

int df_train_num_params(const df_train* t, int64_t* count) {
    if (!t || !count) return set_err(DF_ERR_INVALID, "null pointer");
    *count = t->P;
    return DF_OK;
}

int df_train_sweep(const df_train* t, int* form) {
    if (!t || !form) return set_err(DF_ERR_INVALID, "null pointer");
    if (!t->layerwise) *form = DF_SWEEP_FUSED;
    else if (t->cap == 0)  // no gradient yet: the form ensure_capacity will try first
        *form = t->fmode ? DF_SWEEP_H0FREE
                         : (t->c->plan.uniform || t->sweep_req == DF_SWEEP_RECOMPUTE) ? DF_SWEEP_RECOMPUTE : DF_SWEEP_KEPT;
    else if (t->fmode && t->hsave_on && t->d_fsave) *form = DF_SWEEP_H0FREE;
    else *form = t->hsave_on ? DF_SWEEP_KEPT : DF_SWEEP_RECOMPUTE;
    if (t->layerwise && t->separate) *form |= DF_SWEEP_SEPARATE;
    return DF_OK;
}

int df_train_grad_ptr(df_train* t, float** grad_dev) {
    if (!t || !grad_dev) return set_err(DF_ERR_INVALID, "null pointer");
    *grad_dev = t->d_grad;
    return DF_OK;
}

}  // extern "C"

namespace {
// Whether the kernels normalise θ for this trainer (df_theta_input); DF_THETA_RAW
// without bounds on a conditional chain is an error (-1).
int theta_flow(const df_train* t) {
    const df_chain* c = t->c;
    if (c->plan.n == 0) return 0;
    switch (t->theta_input) {
    case DF_THETA_GIVEN: return 0;
    case DF_THETA_RAW: return c->has_bounds ? 1 : -1;
    default: return c->has_bounds ? 1 : 0;
    }
}
}  // namespace

extern "C" {

int df_train_set_theta_input(df_train* t, int mode) {
    if (!t) return set_err(DF_ERR_INVALID, "null trainer");
    if (mode != DF_THETA_AUTO && mode != DF_THETA_RAW && mode != DF_THETA_GIVEN)
        return set_err(DF_ERR_INVALID, "θ input mode must be DF_THETA_AUTO, DF_THETA_RAW or DF_THETA_GIVEN");
    t->theta_input = mode;
    return DF_OK;
}

int df_train_gradient(df_train* t, const float* x, const float* theta_raw, int64_t batch, int64_t n_total,
                      double* logpdf_sum, void* stream) {
    if (!t) return set_err(DF_ERR_INVALID, "null trainer");
    if (batch < 0) return set_err(DF_ERR_SHAPE, "negative batch size");
    if (n_total < batch || n_total < 1) return set_err(DF_ERR_INVALID, "n_total must be >= batch and >= 1");
    df_chain* c = t->c;
    const Plan& P = c->plan;
    DeviceGuard gd(c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    hipStream_t st = static_cast<hipStream_t>(stream);
    t->last_lp = logpdf_sum ? logpdf_sum : t->d_lpsum;
    t->last_n = n_total;
    if (batch == 0) {
        hipError_t e = hipMemsetAsync(t->d_grad, 0, sizeof(float) * t->P, st);
        if (e == hipSuccess) e = hipMemsetAsync(const_cast<double*>(t->last_lp), 0, sizeof(double), st);
        return e == hipSuccess ? DF_OK : hip_err(e, "hipMemsetAsync");
    }
    if (!x) return set_err(DF_ERR_INVALID, "null input array");
    if (P.n > 0 && !theta_raw)
        return set_err(DF_ERR_SHAPE, "dimensions θ must match (n, dims...) with n number of trained parameters");
    const int tf = theta_flow(t);
    if (tf < 0) return set_err(DF_ERR_INVALID, "θ bounds not set (df_chain_set_theta_bounds) for DF_THETA_RAW");
    const bool flow = tf == 1;
    int rc = ensure_capacity(t, batch);
    if (rc != DF_OK) return rc;

    // 1. inverse pass keeping every layer's output (U[li] = snap[li], U[0] = z)
    const bool fm = t->fmode && t->hsave_on && t->d_fsave;  // H0-free sweep (features + H1 kept)
    rc = run(c, MODE_LOGPDF, flow, x, theta_raw, nullptr, nullptr, nullptr, logpdf_sum ? logpdf_sum : t->d_lpsum,
             batch, stream, t->d_snap, t->hsave_on ? t->d_hsave : nullptr, t->lwidth, fm ? 1 : t->lmax_h,
             fm ? t->d_fsave : nullptr);
    if (rc != DF_OK) return rc;
    const int64_t bd = batch * P.d;
    // 2. z̄ = z / N
    const float inv_n = 1.f / (float)n_total;
    hipError_t e = launch_scale(t->d_zbar, t->d_snap, inv_n, bd, st);
    if (e != hipSuccess) return hip_err(e, "scale kernel launch");
    // 3. reverse sweep, chain order
    if (t->layerwise) {
        rc = lsweep(t, x, theta_raw, batch, inv_n, flow, st);
        if (rc != DF_OK) return rc;
        e = launch_reduce_grads(t->d_partial, t->lgrid, t->P, t->d_grad, st);
        return e == hipSuccess ? DF_OK : hip_err(e, "gradient reduction launch");
    }
    const int64_t ntiles = (batch + 15) / 16;
    const int grid = (int)std::min<int64_t>(t->grid, (ntiles + kTrainWaves - 1) / kTrainWaves);
    for (const SweepOp& op : t->ops) {
        const DevLayer& L = P.layers[op.layer];
        if (op.net < 0) {
            const float* xmn = static_cast<const float*>(c->d_params) + L.norm_off;
            e = launch_norm_adjoint(t->d_zbar, xmn, xmn + P.d, L.alpha, L.beta, P.d, batch, st);
            if (e != hipSuccess) return hip_err(e, "norm adjoint launch");
            continue;
        }
        TrainArgs a{};
        a.u_in = (op.layer + 1 < P.n_layers) ? t->d_snap + (int64_t)(op.layer + 1) * bd : x;
        a.u_out = t->d_snap + (int64_t)op.layer * bd;
        a.theta = theta_raw;
        a.tmin = flow ? c->d_bounds : nullptr;
        a.tmax = flow ? c->d_bounds + P.n : nullptr;
        a.feat = static_cast<const int32_t*>(c->d_tables) + L.feat_tab;
        a.af = static_cast<const int32_t*>(c->d_tables) + L.af_tab;
        a.zbar = t->d_zbar;
        a.ebuf = t->d_ebuf;
        a.partial = t->d_partial;
        a.blob = static_cast<const uint8_t*>(c->d_blob);
        a.tblob = static_cast<const uint8_t*>(t->d_tblob);
        a.sblob = static_cast<const uint8_t*>(c->d_sblob);
        a.tsblob = static_cast<const uint8_t*>(t->d_tsblob);
        a.batch = batch;
        a.p_total = t->P;
        a.d = P.d;
        a.n = P.n;
        a.n_af = L.n_af;
        a.kind = L.kind;
        a.phase = op.phase;
        a.inv_n = inv_n;
        a.net = t->nets[op.net];
        e = launch_train_net(P.ht, t->net_nh[op.net], t->amode, a, (unsigned)grid, t->lds_max, st);
        if (e != hipSuccess) return hip_err(e, "train kernel launch");
    }
    // 4. fixed-order reduction of the workgroup partials
    e = launch_reduce_grads(t->d_partial, grid, t->P, t->d_grad, st);
    return e == hipSuccess ? DF_OK : hip_err(e, "gradient reduction launch");
}

int df_train_apply(df_train* t, void* stream) {
    if (!t) return set_err(DF_ERR_INVALID, "null trainer");
    DeviceGuard gd(t->c->device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (t->debug && t->last_lp) {  // train!(...; debug=true), src/Flows.jl:404-409
        double s = 0.0;
        hipError_t e = hipMemcpyAsync(&s, t->last_lp, sizeof(double), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_err(e, "debug loss read-back");
        const double l = -s / (double)(t->last_n > 0 ? t->last_n : 1);
        if (!std::isfinite(l)) {
            char msg[96];
            std::snprintf(msg, sizeof msg, "non-finite training loss %g: parameters not updated", l);
            return set_err(DF_ERR_NONFINITE, msg);
        }
    }
    hipError_t e = launch_adam(t->d_params, t->d_grad, t->d_m, t->d_v, t->P, t->opt.eta, t->opt.beta1,
                               t->opt.beta2, t->opt.epsilon, t->d_bt, st);
    if (e != hipSuccess) return hip_err(e, "Adam kernel launch");
    return repack(t, st);
}

int df_train_step(df_train* t, const float* x, const float* theta_raw, int64_t batch, double* logpdf_sum,
                  void* stream) {
    if (!t) return set_err(DF_ERR_INVALID, "null trainer");
    if (batch == 0) return DF_OK;
    int rc = df_train_gradient(t, x, theta_raw, batch, batch, logpdf_sum, stream);
    return rc != DF_OK ? rc : df_train_apply(t, stream);
}

int df_train_step_graph(df_train* t, const float* x, const float* theta_raw, int64_t batch, int64_t n_total,
                        double* logpdf_sum, void* stream) {
    if (!t) return set_err(DF_ERR_INVALID, "null trainer");
    if (batch == 0) return DF_OK;
    if (batch < 0) return set_err(DF_ERR_SHAPE, "negative batch size");
    if (n_total < batch) return set_err(DF_ERR_INVALID, "n_total must be >= batch and >= 1");
    DeviceGuard gd(t->c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t now = ++t->use_clock;
    TrainGraph* g = nullptr;
    for (TrainGraph& e : t->graphs)
        if (e.x == x && e.theta == theta_raw && e.lp == logpdf_sum && e.batch == batch && e.n_total == n_total) g = &e;
    if (t->debug) {  // the loss check synchronises: no capture while it is on
        int rc = df_train_gradient(t, x, theta_raw, batch, n_total, logpdf_sum, stream);
        return rc != DF_OK ? rc : df_train_apply(t, stream);
    }
    const int flow_now = theta_flow(t);
    if (g && (g->cap_gen != t->cap_gen || g->partial_gen != t->c->partial_gen ||
              g->flow != flow_now)) {  // stale buffers, or θ now read the other way
        if (g->exec) (void)hipGraphExecDestroy(g->exec);
        g->exec = nullptr;
        g->seen = 0;
    }
    if (g && g->exec) {  // replay
        g->last_use = now;
        hipError_t e = hipGraphLaunch(g->exec, st);
        return e == hipSuccess ? DF_OK : hip_err(e, "hipGraphLaunch(train step)");
    }
    if (!g || g->seen == 0) {  // first sight of this key: eager (allocates every buffer it needs)
        if (!g) {
            if (t->graphs.size() >= 4) {  // keep the 4 most recently used keys
                auto lru = t->graphs.begin();
                for (auto it = t->graphs.begin(); it != t->graphs.end(); ++it)
                    if (it->last_use < lru->last_use) lru = it;
                if (lru->exec) (void)hipGraphExecDestroy(lru->exec);
                t->graphs.erase(lru);
            }
            TrainGraph ng;
            ng.x = x;
            ng.theta = theta_raw;
            ng.lp = logpdf_sum;
            ng.batch = batch;
            ng.n_total = n_total;
            t->graphs.push_back(ng);
            g = &t->graphs.back();
        }
        int rc = df_train_gradient(t, x, theta_raw, batch, n_total, logpdf_sum, stream);
        if (rc == DF_OK) rc = df_train_apply(t, stream);
        g->seen = 1;
        g->flow = flow_now;
        g->cap_gen = t->cap_gen;
        g->partial_gen = t->c->partial_gen;
        g->last_use = now;
        return rc;
    }
    // second sight: capture gradient + Adam + repack on a private stream, then replay
    if (!t->cap_stream && hipStreamCreateWithFlags(&t->cap_stream, hipStreamNonBlocking) != hipSuccess)
        return set_err(DF_ERR_HIP, "hipStreamCreate failed");
    hipError_t e = hipStreamBeginCapture(t->cap_stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) return hip_err(e, "hipStreamBeginCapture");
    int rc = df_train_gradient(t, x, theta_raw, batch, n_total, logpdf_sum, t->cap_stream);
    if (rc == DF_OK) rc = df_train_apply(t, t->cap_stream);
    hipGraph_t graph = nullptr;
    e = hipStreamEndCapture(t->cap_stream, &graph);
    if (rc != DF_OK || e != hipSuccess || !graph) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc != DF_OK ? rc : hip_err(e, "hipStreamEndCapture");
    }
    if (g->cap_gen != t->cap_gen || g->partial_gen != t->c->partial_gen) {  // a buffer moved while capturing
        (void)hipGraphDestroy(graph);
        return set_err(DF_ERR_HIP, "internal: training buffers reallocated during graph capture");
    }
    e = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) {
        g->exec = nullptr;
        return hip_err(e, "hipGraphInstantiate(train step)");
    }
    g->last_use = now;
    e = hipGraphLaunch(g->exec, st);
    return e == hipSuccess ? DF_OK : hip_err(e, "hipGraphLaunch(train step)");
}

int df_train_set_debug(df_train* t, int on) {
    if (!t) return set_err(DF_ERR_INVALID, "null trainer");
    t->debug = on != 0;
    return DF_OK;
}

int df_train_get_params(df_train* t, float* host_out, int64_t count) {
    if (!t || (!host_out && count > 0)) return set_err(DF_ERR_INVALID, "null pointer");
    if (count != t->P) return set_err(DF_ERR_SHAPE, "count must equal df_train_num_params");
    DeviceGuard gd(t->c->device);
    if (count == 0) return DF_OK;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(host_out, t->d_params, sizeof(float) * count, hipMemcpyDeviceToHost);
    return e == hipSuccess ? DF_OK : hip_err(e, "hipMemcpy(params)");
}

int df_train_set_params(df_train* t, const float* host_in, int64_t count) {
    if (!t || (!host_in && count > 0)) return set_err(DF_ERR_INVALID, "null pointer");
    if (count != t->P) return set_err(DF_ERR_SHAPE, "count must equal df_train_num_params");
    DeviceGuard gd(t->c->device);
    if (count == 0) return DF_OK;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(t->d_params, host_in, sizeof(float) * count, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_err(e, "hipMemcpy(params)");
    int rc = repack(t, nullptr);
    if (rc != DF_OK) return rc;
    e = hipDeviceSynchronize();
    return e == hipSuccess ? DF_OK : hip_err(e, "repack");
}

}  // extern "C"

namespace df {
namespace api {
int train_device(const df_train* t) { return t ? t->c->device : -1; }
double* train_last_lpsum(df_train* t) { return t ? const_cast<double*>(t->last_lp) : nullptr; }
}  // namespace api
}  // namespace df
