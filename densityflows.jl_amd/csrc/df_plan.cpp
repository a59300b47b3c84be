// df_plan.cpp — validate a df_chain_desc and pack it for the fused kernels.
//
// Reference semantics restated here (DensityFlows.jl v1.0.0):
//   * conditioner input = vcat(θ, z)[axis_nn]        src/affine/RNVP.jl:157,174,196
//     → the kernel keeps each sample's state row as [θ (n) | z (d) | 0] in LDS,
//       so a 1-based axis_nn entry k is the state slot k-1; padding slot n+d is 0.
//   * x_af = z_af .* exp.(s) .+ t, row k of s/t ↔ dim axis_af[k]   RNVP.jl:182-184
//     → af table: slot n + axis_af[k] - 1.
//   * s/t nets: Chain(Dense(in,h,σ), (n-1)×Dense(h,h,σ), Dense(h,out))  Layers.jl:33-50
//   * Flux.Dense weight is (out, in) column-major: W[i + out*k].
#include "df_plan.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <set>
#include <sstream>

namespace df {
namespace {

struct Fail {
    int code;
    std::string msg;
};

[[noreturn]] void fail(int code, const std::string& m) { throw Fail{code, m}; }

int round_up(int v, int m) { return (v + m - 1) / m * m; }

int pow2_tiles(int t) {
    int p = 1;
    while (p < t) p *= 2;
    return p;
}

// One packable item of a coupling layer, in kernel consumption order.
struct Item {
    enum Kind { CHUNK_KQ, BIAS, W3 } kind;
    int dense;   // index into plan.denses
    int kq;      // CHUNK_KQ: k-quad index
    int bytes;
};

class Packer {
public:
    Packer(Plan& p, int cap) : P(p), cap_(cap) {}

    int remaining() const { return cur_ < 0 ? 0 : cap_ - used_; }
    int cap() const { return cap_; }

    void begin_stage() {
        close();
        cur_ = (int)P.stages.size();
        DevStage s{};
        s.src_off = (int64_t)P.blob.size();
        P.stages.push_back(s);
        used_ = 0;
    }

    // Reserve `bytes` (multiple of 16) in the current stage (opening one if
    // needed).  Returns {stage, byte offset in stage}.
    std::pair<int, int> alloc(int bytes) {
        if (bytes > cap_) fail(DF_ERR_UNSUPPORTED, "packed item exceeds the LDS stage buffer");
        if (cur_ < 0 || used_ + bytes > cap_) begin_stage();
        int off = used_;
        used_ += bytes;
        P.blob.resize((size_t)P.stages[cur_].src_off + used_, 0);
        return {cur_, off};
    }

    float* at(int stage, int off) {
        return reinterpret_cast<float*>(P.blob.data() + P.stages[stage].src_off + off);
    }

    // Pad the open stage to the DMA granularity and record its size.
    void close() {
        if (cur_ >= 0) {
            used_ = round_up(used_, kStageAlign);
            P.blob.resize((size_t)P.stages[cur_].src_off + used_, 0);
            P.stages[cur_].bytes = used_;
            P.stage_max = std::max(P.stage_max, used_);
        }
    }

private:
    Plan& P;
    int cap_;
    int cur_ = -1;
    int used_ = 0;
};

void check_net(const df_dense_desc* net, int nd, int in_dim, int out_dim, const char* which) {
    if (nd < 1) fail(DF_ERR_INVALID, std::string(which) + ": a conditioner needs at least one Dense");
    if (!net) fail(DF_ERR_INVALID, std::string(which) + ": null Dense array");
    int prev = in_dim;
    for (int k = 0; k < nd; ++k) {
        const df_dense_desc& D = net[k];
        if (D.in_dim != prev) {
            std::ostringstream os;
            os << which << ": Dense " << k + 1 << " expects " << D.in_dim << " inputs but receives " << prev;
            fail(DF_ERR_SHAPE, os.str());
        }
        if (D.out_dim < 1 || !D.W) fail(DF_ERR_INVALID, std::string(which) + ": empty Dense");
        if (D.act < DF_ACT_IDENTITY || D.act > DF_ACT_SWISH)
            fail(DF_ERR_INVALID, std::string(which) + ": unknown activation");
        if (k + 1 < nd && D.out_dim > kMaxHidden) fail(DF_ERR_UNSUPPORTED, "hidden width > 256");
        prev = D.out_dim;
    }
    if (prev != out_dim) {
        std::ostringstream os;
        os << which << ": output dimension " << prev << " does not match the " << out_dim
           << " transformed dimensions";
        fail(DF_ERR_SHAPE, os.str());
    }
}

// SPLIT packing of a FAST plan (layout: df_plan.h, kSplit*): every net gets the
// bf16 planes of its first and hidden Dense; nets are packed whole into stages of
// at most max(one net, 24 KiB) (a chain of <= 64 KiB is one stage).  The split
// descriptors are the FAST ones with stage ids and offsets into the split blob.
void build_split(const df_chain_desc* desc, Plan& P, const std::vector<char>& fold) {
    P.split = 0;
    if (!P.fast || (P.ht != 2 && P.ht != 4)) return;
    const int ht = P.ht, H = 16 * ht;
    auto net_bytes = [&](int n_out) {
        return kSplitFirstBytes(ht) + kSplitHiddenBytes(ht) + 4 * H + round_up((n_out * H + 4) * 4, 16);
    };
    int total = 0, biggest = 0;
    for (const ULayer& U : P.ulayers) {
        if (U.kind == DF_LAYER_NORM) continue;
        const int b = net_bytes(U.t.n_out) + (U.kind == DF_LAYER_RNVP ? net_bytes(U.s.n_out) : 0);
        total += b;
        biggest = std::max(biggest, std::max(net_bytes(U.t.n_out), U.kind == DF_LAYER_RNVP ? net_bytes(U.s.n_out) : 0));
    }
    const int cap = total <= kSingleStageCap ? kSingleStageCap : std::max(kStageCap, round_up(biggest, kStageAlign));
    std::vector<uint8_t>& blob = P.sblob;
    int cur = -1, used = 0;
    auto close = [&]() {
        if (cur < 0) return;
        used = round_up(used, kStageAlign);
        blob.resize((size_t)P.sstages[cur].src_off + used, 0);
        P.sstages[cur].bytes = used;
        P.sstage_max = std::max(P.sstage_max, used);
    };
    auto alloc = [&](int bytes) {
        if (cur < 0 || used + bytes > cap) {
            close();
            cur = (int)P.sstages.size();
            DevStage s{};
            s.src_off = (int64_t)blob.size();
            P.sstages.push_back(s);
            used = 0;
        }
        const int off = used;
        used += bytes;
        blob.resize((size_t)P.sstages[cur].src_off + used, 0);
        return std::make_pair(cur, off);
    };
    P.sulayers = P.ulayers;
    for (int li = 0; li < desc->n_layers; ++li) {
        const df_layer_desc& L = desc->layers[li];
        if (L.kind == DF_LAYER_NORM) continue;
        const DevLayer& DL = P.layers[li];
        auto pack = [&](const df_dense_desc* net, int d0, UNet* u) {
            const DevDense &D0 = P.denses[d0], &D1 = P.denses[d0 + 1], &DO = P.denses[d0 + 2];
            auto [st, off] = alloc(net_bytes(u->n_out));
            u->stage = st;
            u->off_w0 = off;
            u->off_h = off + kSplitFirstBytes(ht);
            u->off_out = u->off_h + kSplitHiddenBytes(ht) + 4 * H;
            u->off_b0 = -1;
            u->hstride = 0;
            const int64_t base = P.sstages[st].src_off;
            auto put16 = [&](int64_t at, int32_t src, int plane, float v) {  // at: byte offset in the stage
                const uint16_t h = bf16_split_plane(v, plane);
                std::memcpy(&blob[base + at], &h, 2);
                if (src >= 0) {
                    P.spack_dst.push_back((int32_t)(base + at));
                    P.spack_src.push_back(src * 4 + plane);
                }
            };
            auto put32 = [&](int64_t at, int32_t src, float v) {
                std::memcpy(&blob[base + at], &v, 4);
                if (src >= 0) {
                    P.spack_dst.push_back((int32_t)(base + at));
                    P.spack_src.push_back(src * 4 + 3);
                }
            };
            // first Dense: slots (w0, w0, w1, w0, w1, w2, 0, 0) of W[16m+i, g] (g = 3 folded: the bias)
            const df_dense_desc& W0 = net[0];
            static const int kPlaneOfSlot[6] = {0, 0, 1, 0, 1, 2};
            for (int m = 0; m < ht; ++m)
                for (int lane = 0; lane < 64; ++lane) {
                    const int g = lane >> 4, row = 16 * m + (lane & 15);
                    float v = 0.f;
                    int32_t src = -1;
                    if (row < W0.out_dim) {
                        if (fold[li] && g == 3) {
                            v = W0.b[row];
                            src = D0.b_off + row;
                        } else if (g < W0.in_dim) {
                            v = W0.W[(size_t)row + (size_t)W0.out_dim * g];
                            src = D0.w_off + row + W0.out_dim * g;
                        }
                    }
                    for (int e = 0; e < 6; ++e)
                        put16(u->off_w0 + ((int64_t)m * 64 + lane) * 16 + 2 * e, src, kPlaneOfSlot[e], v);
                }
            // hidden Dense planes
            const df_dense_desc& W1 = net[1];
            for (int c = 0; c < ht / 2; ++c)
                for (int m = 0; m < ht; ++m)
                    for (int p = 0; p < 3; ++p)
                        for (int lane = 0; lane < 64; ++lane)
                            for (int e = 0; e < 8; ++e) {
                                const int g = lane >> 4, row = 16 * m + (lane & 15);
                                const int k = 32 * c + 16 * (e >> 2) + 4 * g + (e & 3);
                                const bool ok = row < W1.out_dim && k < W1.in_dim;
                                put16(u->off_h + ((((int64_t)c * ht + m) * 3 + p) * 64 + lane) * 16 + 2 * e,
                                      ok ? D1.w_off + row + W1.out_dim * k : -1, p,
                                      ok ? W1.W[(size_t)row + (size_t)W1.out_dim * k] : 0.f);
                            }
            const int64_t hb = u->off_h + kSplitHiddenBytes(ht);
            for (int row = 0; row < H; ++row) {
                const bool ok = W1.b && row < W1.out_dim;
                put32(hb + 4 * row, ok ? D1.b_off + row : -1, ok ? W1.b[row] : 0.f);
            }
            // output Dense (VALU GEMV): [o][H] then b[4]
            const df_dense_desc& W2 = net[2];
            for (int o = 0; o < W2.out_dim; ++o)
                for (int k = 0; k < H; ++k) {
                    const bool ok = k < W2.in_dim;
                    put32(u->off_out + 4 * ((int64_t)o * H + k), ok ? DO.w_off + o + W2.out_dim * k : -1,
                          ok ? W2.W[(size_t)o + (size_t)W2.out_dim * k] : 0.f);
                }
            for (int o = 0; o < 4; ++o) {
                const bool ok = W2.b && o < W2.out_dim;
                put32(u->off_out + 4 * ((int64_t)W2.out_dim * H + o), ok ? DO.b_off + o : -1, ok ? W2.b[o] : 0.f);
            }
            P.split_flops_per_sample += 2.0 * (W0.in_dim * W0.out_dim + W1.in_dim * W1.out_dim);
        };
        ULayer& U = P.sulayers[li];
        if (L.kind == DF_LAYER_RNVP) pack(L.s_net, DL.s_dense0, &U.s);
        pack(L.t_net, DL.t_dense0, &U.t);
    }
    close();
    auto sched = [&](bool fwd) {
        std::vector<int32_t> out;
        auto push = [&](int s) {
            if (out.empty() || out.back() != s) out.push_back(s);
        };
        for (int it = 0; it < P.n_layers; ++it) {
            const ULayer& U = P.sulayers[fwd ? it : P.n_layers - 1 - it];
            if (U.kind == DF_LAYER_NORM) continue;
            if (fwd) {
                if (U.kind == DF_LAYER_RNVP) push(U.s.stage);
                push(U.t.stage);
            } else {
                push(U.t.stage);
                if (U.kind == DF_LAYER_RNVP) push(U.s.stage);
            }
        }
        return out;
    };
    P.ssched_fwd = sched(true);
    P.ssched_bwd = sched(false);
    int target = kLdsPerBlockTarget;
    if (const char* e = std::getenv("DF_SPLIT_LDS_KB")) target = std::max(32, std::atoi(e)) * 1024;
    const int nbuf = P.sstages.size() > 1 ? 2 : 1;
    const int fixed = nbuf * P.sstage_max + table_lds_bytes(P);
    const int per_tile = kWavesPerBlock * 16 * P.stride * 4;
    int t = 0;
    while (t < kMaxTilesPerWave && fixed + (t + 1) * per_tile <= target) ++t;
    t -= t % P.tile_group;
    if (t < P.tile_group) {  // no room for one tile group next to the split stages: stay on f32
        P.sulayers.clear();
        P.sstages.clear();
        P.sblob.clear();
        P.spack_dst.clear();
        P.spack_src.clear();
        P.split_flops_per_sample = 0.0;
        return;
    }
    P.stiles = t;
    P.sblob.resize(round_up((int)P.sblob.size(), 16) + 16, 0);
    P.split = 1;
}

// Wide-net packing (see WNet).  Leaves P.wide = 0 unless every coupling layer's
// conditioners are Dense(in <= 64, 256) → Dense(256, 256) → Dense(256, out <= 32).
void build_wide(const df_chain_desc* desc, Plan& P) {
    if (const char* f = std::getenv("DF_NO_WIDE"))
        if (f[0] == '1') return;
    if (P.uniform || P.ht != 16) return;
    for (int li = 0; li < desc->n_layers; ++li) {
        const df_layer_desc& L = desc->layers[li];
        if (L.kind == DF_LAYER_NORM) continue;
        auto ok = [&](const df_dense_desc* net, int nd) {
            return nd == 3 && net[0].in_dim <= kMaxState && net[0].out_dim == 256 && net[1].out_dim == 256 &&
                   net[2].out_dim <= 32 && net[0].act == DF_ACT_RELU && net[1].act == DF_ACT_RELU &&
                   net[2].act == DF_ACT_IDENTITY;
        };
        if (L.kind == DF_LAYER_RNVP && !ok(L.s_net, L.n_dense_s)) return;
        if (!ok(L.t_net, L.n_dense_t)) return;
    }
    int li_dense = 0;  // running index into P.denses (trainables offsets)
    std::vector<WLayer> wl;
    for (int li = 0; li < desc->n_layers; ++li) {
        const df_layer_desc& L = desc->layers[li];
        const DevLayer& DL = P.layers[li];
        WLayer W{};
        W.kind = DL.kind;
        W.elem_start = DL.elem_start;
        W.elem_end = DL.elem_end;
        W.n_af = DL.n_af;
        W.feat_tab = DL.feat_tab;
        W.af_tab = DL.af_tab;
        W.norm_off = DL.norm_off;
        W.alpha = DL.alpha;
        W.beta = DL.beta;
        W.ldj_const = DL.ldj_const;
        if (L.kind != DF_LAYER_NORM) {
            auto pack = [&](const df_dense_desc* net, int d0, WNet& N) {
                const int ks = (net[0].in_dim + 3) / 4;  // state k-steps: feature k = 4s + g
                const int nkq0 = (ks + 3) / 4;
                N.stage0 = (int)P.wstages.size();
                N.nst0 = (nkq0 + 1) / 2;
                N.ks = ks;
                N.n_out = net[2].out_dim;
                N.mto = (N.n_out + 15) / 16;
                N.act0 = net[0].act;
                N.act1 = net[1].act;
                N.act_out = net[2].act;
                auto new_stage = [&](int bytes) -> float* {
                    DevStage st{};
                    st.src_off = (int64_t)P.wblob.size();
                    st.bytes = bytes;
                    P.wstages.push_back(st);
                    P.wblob.resize(P.wblob.size() + bytes, 0);
                    return reinterpret_cast<float*>(P.wblob.data() + st.src_off);
                };
                auto put = [&](float* base, int64_t q, int dense, int row, int k) {
                    const df_dense_desc& D = net[dense];
                    if (row >= D.out_dim || k >= D.in_dim) return;
                    base[q] = D.W[(size_t)row + (size_t)D.out_dim * k];
                    const int64_t f0 = (reinterpret_cast<uint8_t*>(base) - P.wblob.data()) / 4;
                    P.wpack_dst.push_back((int32_t)(f0 + q));
                    P.wpack_src.push_back(P.denses[d0 + dense].w_off + row + D.out_dim * k);
                };
                // first Dense: [kk < 2][m < 16][lane][r], k-step s = 4kq + r, feature 4s + g
                for (int st = 0; st < N.nst0; ++st) {
                    float* b = new_stage(kWideStageBytes);
                    for (int kk = 0; kk < 2; ++kk)
                        for (int m = 0; m < 16; ++m)
                            for (int lane = 0; lane < 64; ++lane)
                                for (int r = 0; r < 4; ++r) {
                                    const int s = 4 * (2 * st + kk) + r;
                                    if (s >= ks) continue;
                                    put(b, ((int64_t)(kk * 16 + m) * 64 + lane) * 4 + r, 0, 16 * m + (lane & 15),
                                        4 * s + (lane >> 4));
                                }
                }
                // hidden Dense: 8 stages of [kk < 2][m < 16], k = 16kq + 4g + r
                for (int st = 0; st < 8; ++st) {
                    float* b = new_stage(kWideStageBytes);
                    for (int kk = 0; kk < 2; ++kk)
                        for (int m = 0; m < 16; ++m)
                            for (int lane = 0; lane < 64; ++lane)
                                for (int r = 0; r < 4; ++r)
                                    put(b, ((int64_t)(kk * 16 + m) * 64 + lane) * 4 + r, 1, 16 * m + (lane & 15),
                                        16 * (2 * st + kk) + 4 * (lane >> 4) + r);
                }
                // output Dense: [kq < 16][m < mto]
                {
                    float* b = new_stage(16 * N.mto * 1024);
                    for (int kq = 0; kq < 16; ++kq)
                        for (int m = 0; m < N.mto; ++m)
                            for (int lane = 0; lane < 64; ++lane)
                                for (int r = 0; r < 4; ++r)
                                    put(b, ((int64_t)(kq * N.mto + m) * 64 + lane) * 4 + r, 2, 16 * m + (lane & 15),
                                        16 * kq + 4 * (lane >> 4) + r);
                }
                // every wide Dense gets a bias row (zeros without a bias: the kernel adds it
                // unconditionally, no per-element select; x + 0 = x up to the sign of a zero)
                auto bias = [&](int dense, int rows) -> int32_t {
                    const df_dense_desc& D = net[dense];
                    const int32_t off = (int32_t)P.wbias.size();
                    P.wbias.resize(P.wbias.size() + rows, 0.f);
                    if (!D.b) return off;
                    for (int r = 0; r < D.out_dim; ++r) {
                        P.wbias[off + r] = D.b[r];
                        P.wbias_dst.push_back(off + r);
                        P.wbias_src.push_back(P.denses[d0 + dense].b_off + r);
                    }
                    return off;
                };
                N.b0 = bias(0, 256);
                N.b1 = bias(1, 256);
                N.bo = bias(2, 16 * N.mto);
            };
            if (L.kind == DF_LAYER_RNVP) pack(L.s_net, DL.s_dense0, W.s);
            pack(L.t_net, DL.t_dense0, W.t);
        }
        wl.push_back(W);
    }
    (void)li_dense;
    auto sched = [&](bool fwd) {
        std::vector<int32_t> out;
        auto net = [&](const WNet& N) {
            for (int s = 0; s < N.nst0 + 9; ++s) out.push_back(N.stage0 + s);
        };
        for (int it = 0; it < P.n_layers; ++it) {
            const WLayer& L = wl[fwd ? it : P.n_layers - 1 - it];
            if (L.kind == DF_LAYER_NORM) continue;
            if (fwd) {
                if (L.kind == DF_LAYER_RNVP) net(L.s);
                net(L.t);
            } else {
                net(L.t);
                if (L.kind == DF_LAYER_RNVP) net(L.s);
            }
        }
        return out;
    };
    P.wsched_fwd = sched(true);
    P.wsched_bwd = sched(false);
    P.wlayers = std::move(wl);
    P.wblob.resize(P.wblob.size() + 16, 0);
    P.wbias.resize(P.wbias.size() + 4, 0.f);
    P.wide = 1;
}

// SPLIT packing of a wide plan (see Plan::wsplit): per net, ceil(in/32) first-Dense
// stages, 8 hidden stages, one output stage, each chunk [m][plane][lane][8 bf16]
// with lane (g, i) holding W[16m + i, k(e)], e < 8:
//   first Dense  k = 32c + 8g + e (features through the layer's split table)
//   hidden/out   k = 32c + 16(e>>2) + 4g + (e&3) (accumulator tiles 2c, 2c+1)
void build_wide_split(const df_chain_desc* desc, Plan& P) {
    P.wsplit = 0;
    if (!P.wide) return;
    P.wstables = P.tables;
    P.wslayers = P.wlayers;
    const int zero_slot = P.n + P.d;
    for (int li = 0; li < desc->n_layers; ++li) {
        const df_layer_desc& L = desc->layers[li];
        if (L.kind == DF_LAYER_NORM) continue;
        const DevLayer& DL = P.layers[li];
        WLayer& W = P.wslayers[li];
        const int nc0 = (L.n_nn + 31) / 32;
        W.pad0 = (int32_t)P.wstables.size();
        for (int k = 0; k < 32 * nc0; ++k) P.wstables.push_back(k < L.n_nn ? L.axis_nn[k] - 1 : zero_slot);
        auto pack = [&](const df_dense_desc* net, int d0, WNet& N) {
            N.stage0 = (int)P.wsstages.size();
            N.nst0 = nc0 * kWideSplitHalves;
            N.nso = (kWideSplitHalves == 2 && N.mto == 2) ? 2 : 1;
            auto new_stage = [&](int bytes) -> int64_t {
                DevStage st{};
                st.src_off = (int64_t)P.wsblob.size();
                st.bytes = bytes;
                P.wsstages.push_back(st);
                P.wsblob.resize(P.wsblob.size() + bytes, 0);
                return st.src_off;
            };
            // chunk [m < mt][plane][lane][8] of m-tiles m0 + m at byte `base` of the blob, k(c, g, e) as above
            auto chunk = [&](int64_t base, int dense, int c, int mt, bool first, int m0 = 0) {
                const df_dense_desc& D = net[dense];
                for (int m = 0; m < mt; ++m)
                    for (int p = 0; p < 3; ++p)
                        for (int lane = 0; lane < 64; ++lane)
                            for (int e = 0; e < 8; ++e) {
                                const int g = lane >> 4, row = 16 * (m0 + m) + (lane & 15);
                                const int k = first ? 32 * c + 8 * g + e : 32 * c + 16 * (e >> 2) + 4 * g + (e & 3);
                                const int64_t at = base + (((int64_t)m * 3 + p) * 64 + lane) * 16 + 2 * e;
                                uint16_t h = 0;
                                if (row < D.out_dim && k < D.in_dim) {
                                    h = bf16_split_plane(D.W[(size_t)row + (size_t)D.out_dim * k], p);
                                    P.wspack_dst.push_back((int32_t)at);
                                    P.wspack_src.push_back((P.denses[d0 + dense].w_off + row + D.out_dim * k) * 4 + p);
                                }
                                std::memcpy(&P.wsblob[at], &h, 2);
                            }
            };
            constexpr int MH = 16 / kWideSplitHalves;  // m-tiles per stage
            for (int c = 0; c < nc0; ++c)
                for (int hv = 0; hv < kWideSplitHalves; ++hv)
                    chunk(new_stage(kWideSplitStageBytes), 0, c, MH, true, MH * hv);
            for (int c = 0; c < 8; ++c)
                for (int hv = 0; hv < kWideSplitHalves; ++hv)
                    chunk(new_stage(kWideSplitStageBytes), 1, c, MH, false, MH * hv);
            const int cps = 8 / N.nso;  // output chunks per stage
            for (int so = 0; so < N.nso; ++so) {
                const int64_t ob = new_stage(cps * N.mto * 3 * 1024);
                for (int c = 0; c < cps; ++c) chunk(ob + (int64_t)c * N.mto * 3 * 1024, 2, so * cps + c, N.mto, false);
            }
            P.split_flops_per_sample += 2.0 * ((double)net[0].in_dim * net[0].out_dim +
                                               (double)net[1].in_dim * net[1].out_dim +
                                               (double)net[2].in_dim * net[2].out_dim);
        };
        if (L.kind == DF_LAYER_RNVP) pack(L.s_net, DL.s_dense0, W.s);
        pack(L.t_net, DL.t_dense0, W.t);
    }
    auto sched = [&](bool fwd) {
        std::vector<int32_t> out;
        auto net = [&](const WNet& N) {
            for (int s = 0; s < N.nst0 + 8 * kWideSplitHalves + N.nso; ++s) out.push_back(N.stage0 + s);
        };
        for (int it = 0; it < P.n_layers; ++it) {
            const WLayer& L = P.wslayers[fwd ? it : P.n_layers - 1 - it];
            if (L.kind == DF_LAYER_NORM) continue;
            if (fwd) {
                if (L.kind == DF_LAYER_RNVP) net(L.s);
                net(L.t);
            } else {
                net(L.t);
                if (L.kind == DF_LAYER_RNVP) net(L.s);
            }
        }
        return out;
    };
    P.wssched_fwd = sched(true);
    P.wssched_bwd = sched(false);
    P.wsblob.resize(P.wsblob.size() + 16, 0);
    P.wsplit = 1;
}

}  // namespace

size_t plan_lds_bytes(const Plan& p) {
    size_t tab = (size_t)table_lds_bytes(p);
    const int nbuf = p.stages.size() > 1 ? 2 : 1;
    return (size_t)nbuf * p.stage_max + tab + (size_t)p.samples_per_block * p.stride * 4;
}

int build_plan(const df_chain_desc* desc, Plan* out, std::string* err, int exact) {
    try {
        if (!desc || !out) fail(DF_ERR_INVALID, "null descriptor");
        // the descriptor structs are unchanged since ABI 2 (ABI 3 added entry points only)
        if (desc->abi_version < 2 || desc->abi_version > DF_ABI_VERSION) fail(DF_ERR_INVALID, "ABI version mismatch");
        const int d = desc->d, n = desc->n;
        if (d < 1 || n < 0) fail(DF_ERR_INVALID, "d must be >= 1 and n >= 0");
        if (n + d > kMaxState) fail(DF_ERR_UNSUPPORTED, "n + d > 64 is outside the fused kernel's limits");
        if (desc->n_layers < 1 || !desc->layers) fail(DF_ERR_INVALID, "a FlowChain needs at least one element");
        if (desc->n_layers > kMaxLayers) fail(DF_ERR_UNSUPPORTED, "too many layers");

        Plan P;
        P.d = d;
        P.n = n;
        P.n_layers = desc->n_layers;
        P.stride = n + d + 3;                 // [θ | z | 0 | ldj_chain | ldj_elem]
        if (P.stride % 2 == 0) P.stride += 1; // odd stride: spread LDS banks

        // ---------- pass 0: output path of the conditioner nets ----------
        // A final Dense with <= 4 outputs after >= 1 hidden Dense is evaluated as a
        // VALU GEMV (kernel variant OUTV); the choice is chain-wide.
        bool all_valu = true;
        for (int li = 0; li < desc->n_layers; ++li) {
            const df_layer_desc& L = desc->layers[li];
            if (L.kind == DF_LAYER_NORM) continue;
            const bool ok = (L.kind == DF_LAYER_NICE || L.n_dense_s >= 2) && L.n_dense_t >= 2 && L.n_af <= 4;
            all_valu = all_valu && ok;
        }
        P.outv = all_valu ? 1 : 0;

        // ---------- pass 1: validation, kernel variant (row tiles) ----------
        int max_tiles = 1;
        for (int li = 0; li < desc->n_layers; ++li) {
            const df_layer_desc& L = desc->layers[li];
            if (li > 0 && L.element < desc->layers[li - 1].element)
                fail(DF_ERR_INVALID, "layer element indices must be non-decreasing");
            if (L.kind == DF_LAYER_NORM) {
                if (!L.x_min || !L.x_max) fail(DF_ERR_INVALID, "NormalizationLayer without x_min/x_max");
                if (!(L.beta > L.alpha))
                    fail(DF_ERR_INVALID, "Bounds of the normalisation need to be in the correct order, β > α.");
                continue;
            }
            if (L.kind != DF_LAYER_RNVP && L.kind != DF_LAYER_NICE) fail(DF_ERR_INVALID, "unknown layer kind");
            if (L.n_af < 1 || L.n_af > d || !L.axis_af) fail(DF_ERR_INVALID, "invalid axis_af");
            if (L.n_af > kMaxAf) fail(DF_ERR_UNSUPPORTED, "more than 32 transformed dims in one layer");
            std::set<int> seen;
            for (int k = 0; k < L.n_af; ++k) {
                int a = L.axis_af[k];
                if (a < 1 || a > d) fail(DF_ERR_INVALID, "The mask cannot contain values higher than the dimension");
                if (!seen.insert(a).second) fail(DF_ERR_INVALID, "axis_af contains a repeated dimension");
            }
            if (L.n_nn < 1 || L.n_nn > n + d || !L.axis_nn) fail(DF_ERR_INVALID, "invalid axis_nn");
            for (int k = 0; k < L.n_nn; ++k) {
                if (L.axis_nn[k] < 1 || L.axis_nn[k] > n + d) fail(DF_ERR_INVALID, "axis_nn out of range");
                // the conditioner must not read transformed dims (else the layer is not a coupling)
                if (L.axis_nn[k] > n && seen.count(L.axis_nn[k] - n))
                    fail(DF_ERR_UNSUPPORTED, "axis_nn contains a transformed dimension");
            }
            if (L.kind == DF_LAYER_RNVP) {
                check_net(L.s_net, L.n_dense_s, L.n_nn, L.n_af, "s_net");
            } else if (L.n_dense_s != 0) {
                fail(DF_ERR_INVALID, "NICECouplingLayer has no s_net");
            }
            check_net(L.t_net, L.n_dense_t, L.n_nn, L.n_af, "t_net");
            auto scan = [&](const df_dense_desc* net, int nd) {
                for (int k = 0; k < nd; ++k) {
                    bool last = (k + 1 == nd);
                    bool valu_last = last && all_valu;
                    if (!valu_last) max_tiles = std::max(max_tiles, (net[k].out_dim + 15) / 16);
                    if (k > 0) max_tiles = std::max(max_tiles, (net[k].in_dim + 15) / 16);
                }
            };
            if (L.kind == DF_LAYER_RNVP) scan(L.s_net, L.n_dense_s);
            scan(L.t_net, L.n_dense_t);
        }
        P.ht = pow2_tiles(max_tiles);
        if (P.ht > kMaxHidden / 16) fail(DF_ERR_UNSUPPORTED, "hidden width > 256");

        // ---------- pass 1b: does every net have the default _dflt_net shape? ----------
        // Dense(in<=16, H) -> nh × Dense(H, H) -> Dense(H, out) with ceil(H/16) = HT <= 4,
        // one hidden σ per net.  Such chains run on the specialised kernel, whose
        // first Dense uses a compact fragment layout (no k-quad padding).
        bool uniform_shape = P.ht <= 4;
        bool relu_only = true;
        if (const char* f = std::getenv("DF_FORCE_GENERIC"))
            if (f[0] == '1') uniform_shape = false;
        for (int li = 0; li < desc->n_layers && uniform_shape; ++li) {
            const df_layer_desc& L = desc->layers[li];
            if (L.kind == DF_LAYER_NORM) continue;
            auto ok_net = [&](const df_dense_desc* net, int nd) {
                if (nd < 2 || (L.n_nn + 3) / 4 > 4) return false;
                for (int k = 0; k + 1 < nd; ++k) {
                    if ((net[k].out_dim + 15) / 16 != P.ht) return false;
                    if (k >= 1 && net[k].act != net[1].act) return false;
                    if (net[k].act != DF_ACT_RELU) relu_only = false;
                }
                if (net[nd - 1].act != DF_ACT_IDENTITY) relu_only = false;
                if (!all_valu && (net[nd - 1].out_dim + 15) / 16 > 2) return false;
                return true;
            };
            if (L.kind == DF_LAYER_RNVP) uniform_shape = uniform_shape && ok_net(L.s_net, L.n_dense_s);
            uniform_shape = uniform_shape && ok_net(L.t_net, L.n_dense_t);
        }

        // ---------- pass 1c: first-Dense bias folding (specialised kernel) ----------
        // With in < 4·ks the compact first Dense has a free k-slot; the LAST one
        // (k = 4·ks − 1) carries the bias against a state column that holds 1, so the
        // MFMA chain ends with fma(b, 1, Σ_k W x) = round(W*x + b): bit-identical to
        // the separate `W*x .+ b` (Flux) add it replaces.  Both nets of a layer share
        // the feature table, so a layer folds only when all of its nets have a bias.
        std::vector<char> fold(desc->n_layers, 0);
        bool allow_fold = uniform_shape, fold_all = true, any_fold = false, ks1_all = true;
        if (const char* e = std::getenv("DF_NO_FOLD"))
            if (e[0] == '1') allow_fold = false;
        for (int li = 0; li < desc->n_layers; ++li) {
            const df_layer_desc& L = desc->layers[li];
            if (L.kind == DF_LAYER_NORM) continue;
            const int ks = (L.n_nn + 3) / 4;
            const bool f = allow_fold && L.n_nn < 4 * ks && L.t_net[0].b != nullptr &&
                           (L.kind != DF_LAYER_RNVP || L.s_net[0].b != nullptr);
            fold[li] = f ? 1 : 0;
            any_fold = any_fold || f;
            fold_all = fold_all && f;
            ks1_all = ks1_all && ks == 1;
        }
        const int one_slot = n + d + 3;
        if (any_fold) {  // [θ | z | 0 | ldj_chain | ldj_elem | 1]
            P.stride = n + d + 4;
            if (P.stride % 2 == 0) P.stride += 1;
        }

        // ---------- pass 2: packing ----------
        // Whole chain in one stage when it is small (loaded once per workgroup);
        // otherwise 24 KiB stages, double-buffered in LDS, one net per stage
        // whenever a net fits.
        int64_t total_bytes = 0;
        for (int li = 0; li < desc->n_layers; ++li) {
            const df_layer_desc& L = desc->layers[li];
            if (L.kind == DF_LAYER_NORM) continue;
            auto net_bytes = [&](const df_dense_desc* net, int nd) {
                int64_t b = 0;
                int prev_tiles = 0;
                for (int k = 0; k < nd; ++k) {
                    const bool last = (k + 1 == nd);
                    if (last && all_valu) {
                        b += round_up((net[k].out_dim * 16 * prev_tiles + 4) * 4, 16);
                    } else {
                        const int mt = (net[k].out_dim + 15) / 16;
                        const int ks = (k == 0) ? (L.n_nn + 3) / 4 : 4 * prev_tiles;
                        if (k == 0 && uniform_shape) b += (int64_t)mt * ks * 256 + mt * 64;
                        else b += (int64_t)((ks + 3) / 4) * mt * 1024 + mt * 64;
                        prev_tiles = mt;
                    }
                }
                return b;
            };
            if (L.kind == DF_LAYER_RNVP) total_bytes += net_bytes(L.s_net, L.n_dense_s);
            total_bytes += net_bytes(L.t_net, L.n_dense_t);
        }
        // Wide conditioners (>= 128 hidden) run one 16-sample tile per wave, so the
        // stage-switch barrier is amortised over the MFMAs of one stage: give them
        // the largest stages that still fit twice next to the state tile.
        int cap = kStageCap;
        if (P.ht >= 8 && !uniform_shape) {
            int tab_ints = 0;
            for (int li = 0; li < desc->n_layers; ++li)
                if (desc->layers[li].kind != DF_LAYER_NORM)
                    tab_ints += 4 * ((desc->layers[li].n_nn + 3) / 4) + desc->layers[li].n_af;
            const int state = kWavesPerBlock * 16 * P.stride * 4;
            const int room = (160 * 1024 - state - round_up(tab_ints * 4, 16) - 1024) / 2;
            cap = std::max(kStageCap, std::min(kBigStageCap, room / kStageAlign * kStageAlign));
        }
        if (const char* e = std::getenv("DF_STAGE_KB")) cap = std::max(4, std::atoi(e)) * 1024;
        Packer pk(P, total_bytes <= kSingleStageCap ? kSingleStageCap : cap);
        const int zero_slot = n + d;
        for (int li = 0; li < desc->n_layers; ++li) {
            const df_layer_desc& L = desc->layers[li];
            DevLayer DL{};
            DL.kind = L.kind;
            DL.elem_start = (li == 0 || desc->layers[li - 1].element != L.element) ? 1 : 0;
            DL.elem_end = (li + 1 == desc->n_layers || desc->layers[li + 1].element != L.element) ? 1 : 0;

            if (L.kind == DF_LAYER_NORM) {
                DL.norm_off = (int)P.params.size();
                for (int i = 0; i < d; ++i) P.params.push_back(L.x_min[i]);
                for (int i = 0; i < d; ++i) P.params.push_back(L.x_max[i]);
                DL.alpha = L.alpha;
                DL.beta = L.beta;
                // ldj = sum(log.(x_diff ./ δ)) in Float32, sequential (Base.sum, n < 16)
                // src/norm/Normalization.jl:88
                const float delta = L.beta - L.alpha;
                float acc = 0.f;
                for (int i = 0; i < d; ++i) {
                    float xd = L.x_max[i] - L.x_min[i];
                    float v = logf(xd / delta);
                    acc = (i == 0) ? v : acc + v;
                }
                DL.ldj_const = acc;
                P.layers.push_back(DL);
                continue;
            }

            DL.n_af = L.n_af;
            const int ks_state = (L.n_nn + 3) / 4;
            // feature table [ks*4]: k = 4s + g → state slot of vcat(θ,z)[axis_nn[k]]
            DL.feat_tab = (int)P.tables.size();
            for (int k = 0; k < ks_state * 4; ++k)
                P.tables.push_back(k < L.n_nn ? L.axis_nn[k] - 1
                                              : (fold[li] && k == 4 * ks_state - 1) ? one_slot : zero_slot);
            DL.af_tab = (int)P.tables.size();
            for (int k = 0; k < L.n_af; ++k) P.tables.push_back(n + L.axis_af[k] - 1);

            const bool valu = all_valu;
            DL.out_valu = valu ? 1 : 0;

            // Create DevDense entries and the item list for this layer.
            std::vector<Item> items;
            auto add_net = [&](const df_dense_desc* net, int nd, int32_t* first, int32_t* count) {
                *first = (int)P.denses.size();
                *count = nd;
                int prev_tiles = 0;
                for (int k = 0; k < nd; ++k) {
                    const df_dense_desc& D = net[k];
                    DevDense DD{};
                    DD.in_kind = (k == 0) ? IN_STATE : IN_HIDDEN;
                    DD.n_out = D.out_dim;
                    DD.in_dim = D.in_dim;
                    DD.act = D.act;
                    DD.has_bias = D.b ? 1 : 0;
                    DD.out_valu = (k + 1 == nd) && valu ? 1 : 0;
                    if (DD.in_kind == IN_STATE) {
                        DD.ks = ks_state;
                        DD.kt_in = 0;
                    } else {
                        DD.kt_in = prev_tiles;
                        DD.ks = 4 * prev_tiles;
                    }
                    DD.mt = DD.out_valu ? 0 : (D.out_dim + 15) / 16;
                    prev_tiles = DD.mt;
                    DD.w_off = (int32_t)P.trainables.size();
                    for (int64_t q = 0; q < (int64_t)D.in_dim * D.out_dim; ++q) P.trainables.push_back(D.W[q]);
                    DD.b_off = -1;
                    if (D.b) {
                        DD.b_off = (int32_t)P.trainables.size();
                        for (int q = 0; q < D.out_dim; ++q) P.trainables.push_back(D.b[q]);
                    }
                    int idx = (int)P.denses.size();
                    P.denses.push_back(DD);
                    if (DD.out_valu) {
                        items.push_back({Item::W3, idx, 0, round_up((D.out_dim * 16 * DD.kt_in + 4) * 4, 16)});
                    } else if (DD.in_kind == IN_STATE && uniform_shape) {
                        P.denses[idx].compact = 1;
                        items.push_back({Item::CHUNK_KQ, idx, 0, round_up(DD.mt * DD.ks * 256, 16)});
                        items.push_back({Item::BIAS, idx, 0, DD.mt * 16 * 4});
                    } else {
                        int nkq = (DD.ks + 3) / 4;
                        for (int kq = 0; kq < nkq; ++kq) items.push_back({Item::CHUNK_KQ, idx, kq, DD.mt * 1024});
                        items.push_back({Item::BIAS, idx, 0, DD.mt * 16 * 4});
                    }
                }
            };
            if (L.kind == DF_LAYER_RNVP) add_net(L.s_net, L.n_dense_s, &DL.s_dense0, &DL.s_ndense);
            else { DL.s_dense0 = 0; DL.s_ndense = 0; }
            add_net(L.t_net, L.n_dense_t, &DL.t_dense0, &DL.t_ndense);

            // Keep a layer — else each net — inside one stage whenever it fits.
            int layer_bytes = 0;
            for (auto& it : items) layer_bytes += it.bytes;
            if (layer_bytes > pk.remaining() && layer_bytes <= pk.cap()) pk.begin_stage();
            const int t_first_dense = DL.t_dense0;
            auto net_bytes_from = [&](size_t i0) {
                int b = 0;
                for (size_t i = i0; i < items.size(); ++i) {
                    if ((items[i].dense >= t_first_dense) != (items[i0].dense >= t_first_dense)) break;
                    b += items[i].bytes;
                }
                return b;
            };

            // dense index → source Dense for packing
            auto src_of = [&](int dense_idx) -> const df_dense_desc& {
                if (L.kind == DF_LAYER_RNVP && dense_idx < DL.s_dense0 + DL.s_ndense)
                    return L.s_net[dense_idx - DL.s_dense0];
                return L.t_net[dense_idx - DL.t_dense0];
            };

            for (size_t ii = 0; ii < items.size(); ++ii) {
                const Item& it = items[ii];
                const bool net_start = (ii == 0) || ((items[ii - 1].dense >= t_first_dense) != (it.dense >= t_first_dense));
                if (net_start) {
                    const int nb = net_bytes_from(ii);
                    if (nb > pk.remaining() && nb <= pk.cap()) pk.begin_stage();
                }
                DevDense& DD = P.denses[it.dense];
                const df_dense_desc& D = src_of(it.dense);
                const int out = D.out_dim, in = D.in_dim;
                auto [st, off] = pk.alloc(it.bytes);
                float* dst = pk.at(st, off);
                const int64_t dst0 = (P.stages[st].src_off + off) / 4;  // blob float index of dst[0]
                // W(row, k) at dst[q]: value, and the index map for device-side repacking
                auto Wp = [&](float* at, int row, int k) {
                    if (row < out && k < in) {
                        *at = D.W[(size_t)row + (size_t)out * k];
                        P.pack_dst.push_back((int32_t)(dst0 + (at - dst)));
                        P.pack_src.push_back(DD.w_off + row + out * k);
                    } else {
                        *at = 0.f;
                    }
                };
                auto Bp = [&](float* at, int row) {
                    if (D.b && row < out) {
                        *at = D.b[row];
                        P.pack_dst.push_back((int32_t)(dst0 + (at - dst)));
                        P.pack_src.push_back(DD.b_off + row);
                    } else {
                        *at = 0.f;
                    }
                };
                if (it.kind == Item::CHUNK_KQ) {
                    // merge with the previous chunk of this dense when contiguous in the same stage
                    if (DD.n_chunks > 0) {
                        DevChunk& C = P.chunks[DD.chunk0 + DD.n_chunks - 1];
                        if (C.stage == st && C.lds_off + (C.kq_end - C.kq_begin) * DD.mt * 1024 == off &&
                            C.kq_end == it.kq) {
                            C.kq_end++;
                        } else {
                            P.chunks.push_back({st, off, it.kq, it.kq + 1});
                            DD.n_chunks++;
                        }
                    } else {
                        DD.chunk0 = (int)P.chunks.size();
                        P.chunks.push_back({st, off, it.kq, it.kq + 1});
                        DD.n_chunks = 1;
                    }
                    if (DD.compact) {  // [m][r < ks][lane]: k = 4r + g
                        for (int m = 0; m < DD.mt; ++m)
                            for (int r = 0; r < DD.ks; ++r)
                                for (int lane = 0; lane < 64; ++lane) {
                                    const int k = 4 * r + (lane >> 4), row = 16 * m + (lane & 15);
                                    float* at = &dst[(m * DD.ks + r) * 64 + lane];
                                    if (fold[li] && k == 4 * DD.ks - 1) Bp(at, row);  // bias · state[one_slot]
                                    else Wp(at, row, k);
                                }
                        continue;
                    }
                    // fragment [m][lane][r] for k-quad kq
                    for (int m = 0; m < DD.mt; ++m)
                        for (int lane = 0; lane < 64; ++lane)
                            for (int r = 0; r < 4; ++r) {
                                const int i = lane & 15, g = lane >> 4;
                                const int s = 4 * it.kq + r;
                                const int row = 16 * m + i;
                                int k;
                                if (DD.in_kind == IN_STATE) k = (s < DD.ks) ? 4 * s + g : in;  // beyond in → 0
                                else k = 16 * it.kq + 4 * g + r;
                                Wp(&dst[(m * 64 + lane) * 4 + r], row, k);
                            }
                } else if (it.kind == Item::BIAS) {
                    DD.bias_stage = st;
                    DD.bias_lds = off;
                    for (int row = 0; row < DD.mt * 16; ++row) Bp(&dst[row], row);
                } else {  // W3: VALU GEMV output  [o][16*kt_in] then b[4]
                    DD.w3_stage = st;
                    DD.w3_lds = off;
                    const int inp = 16 * DD.kt_in;
                    for (int o = 0; o < out; ++o)
                        for (int k = 0; k < inp; ++k) Wp(&dst[o * inp + k], o, k);
                    for (int o = 0; o < 4; ++o) Bp(&dst[out * inp + o], o);
                }
                (void)in;
            }
            P.layers.push_back(DL);

            // bookkeeping: parameters and algorithmic FLOPs (2 × MACs)
            auto count = [&](const df_dense_desc* net, int nd) {
                for (int k = 0; k < nd; ++k) {
                    P.n_params += (int64_t)net[k].in_dim * net[k].out_dim + (net[k].b ? net[k].out_dim : 0);
                    P.flops_per_sample += 2.0 * net[k].in_dim * net[k].out_dim;
                }
            };
            if (L.kind == DF_LAYER_RNVP) count(L.s_net, L.n_dense_s);
            count(L.t_net, L.n_dense_t);
        }
        pk.close();

        // Stage schedules: the order in which the kernel's ensure_stage() calls
        // ask for stages (forward: s-net then t-net per layer; inverse: layers
        // reversed, t-net then s-net), consecutive duplicates removed.
        auto sched = [&](bool fwd) {
            std::vector<int32_t> out;
            auto push = [&](int s) {
                if (out.empty() || out.back() != s) out.push_back(s);
            };
            auto net = [&](int d0, int nd) {
                for (int k = 0; k < nd; ++k) {
                    const DevDense& D = P.denses[d0 + k];
                    if (D.out_valu) {
                        push(D.w3_stage);
                    } else {
                        for (int c = 0; c < D.n_chunks; ++c) push(P.chunks[D.chunk0 + c].stage);
                        push(D.bias_stage);
                    }
                }
            };
            for (int it = 0; it < P.n_layers; ++it) {
                const DevLayer& L = P.layers[fwd ? it : P.n_layers - 1 - it];
                if (L.kind == DF_LAYER_NORM) continue;
                if (fwd) {
                    net(L.s_dense0, L.s_ndense);
                    net(L.t_dense0, L.t_ndense);
                } else {
                    net(L.t_dense0, L.t_ndense);
                    net(L.s_dense0, L.s_ndense);
                }
            }
            return out;
        };
        P.sched_fwd = sched(true);
        P.sched_bwd = sched(false);

        // Tiles of 16 samples per wave kept resident in LDS.  When every net lives
        // in one stage, a stage switch serves all of a wave's tiles, so take as
        // many as fit two workgroups per CU (<= 80 KiB each); otherwise one tile.
        bool resident = true;
        for (const DevLayer& L : P.layers) {
            if (L.kind == DF_LAYER_NORM) continue;
            auto one_stage = [&](int d0, int nd) {
                int st = -1;
                for (int k = 0; k < nd; ++k) {
                    const DevDense& D = P.denses[d0 + k];
                    std::vector<int> ss;
                    if (D.out_valu) ss.push_back(D.w3_stage);
                    else {
                        for (int c = 0; c < D.n_chunks; ++c) ss.push_back(P.chunks[D.chunk0 + c].stage);
                        ss.push_back(D.bias_stage);
                    }
                    for (int x : ss) {
                        if (st < 0) st = x;
                        if (x != st) return false;
                    }
                }
                return true;
            };
            resident = resident && one_stage(L.s_dense0, L.s_ndense) && one_stage(L.t_dense0, L.t_ndense);
        }
        // Specialised-kernel descriptors when every net has the default shape.
        P.uniform = (uniform_shape && resident) ? 1 : 0;
        P.relu_only = (P.uniform && relu_only) ? 1 : 0;
        bool nh1_all = true;  // every conditioner has exactly one hidden H×H Dense (n_sublayers = 2)
        for (int li = 0; li < desc->n_layers; ++li) {
            const df_layer_desc& L = desc->layers[li];
            if (L.kind == DF_LAYER_NORM) continue;
            nh1_all = nh1_all && L.n_dense_t == 3 && (L.kind != DF_LAYER_RNVP || L.n_dense_s == 3);
        }
        P.fast = (P.relu_only && allow_fold && fold_all && ks1_all && nh1_all) ? 1 : 0;
        if (const char* f = std::getenv("DF_NO_FAST"))
            if (f[0] == '1') P.fast = 0;
        if (uniform_shape && !resident) fail(DF_ERR_UNSUPPORTED, "internal: default-shape net split across stages");
        auto make_unet = [&](int d0, int nd, UNet* u) -> bool {
            if (nd < 2) return false;
            const DevDense& D0 = P.denses[d0];
            if (D0.in_kind != IN_STATE || D0.ks > 4 || D0.mt != P.ht || D0.n_chunks != 1 || !D0.compact) return false;
            const DevChunk& C0 = P.chunks[D0.chunk0];
            u->stage = C0.stage;
            u->ks = D0.ks;
            u->nh = nd - 2;
            u->off_w0 = C0.lds_off;
            u->off_b0 = D0.bias_lds;
            u->act0 = D0.act;
            u->acth = DF_ACT_IDENTITY;
            u->hstride = P.ht * P.ht * 1024 + 64 * P.ht;
            for (int k = 1; k + 1 < nd; ++k) {
                const DevDense& D = P.denses[d0 + k];
                if (D.mt != P.ht || D.kt_in != P.ht || D.n_chunks != 1) return false;
                const DevChunk& C = P.chunks[D.chunk0];
                if (C.kq_begin != 0 || C.kq_end != P.ht) return false;
                if (k == 1) {
                    u->off_h = C.lds_off;
                    u->acth = D.act;
                }
                if (D.act != u->acth) return false;
                if (C.lds_off != u->off_h + (k - 1) * u->hstride) return false;
                if (D.bias_lds != C.lds_off + P.ht * P.ht * 1024) return false;
            }
            if (nd == 2) u->off_h = 0;
            const DevDense& DL = P.denses[d0 + nd - 1];
            if (DL.kt_in != P.ht) return false;
            u->n_out = DL.n_out;
            u->act_out = DL.act;
            if (DL.out_valu) {
                u->off_out = DL.w3_lds;
            } else {
                if (DL.n_chunks != 1) return false;
                const DevChunk& C = P.chunks[DL.chunk0];
                if (C.kq_begin != 0 || C.kq_end != P.ht) return false;
                u->off_out = C.lds_off;
                if (DL.bias_lds != C.lds_off + P.ht * DL.mt * 1024) return false;
            }
            return true;
        };
        if (P.uniform) {
            for (const DevLayer& L : P.layers) {
                ULayer U{};
                U.kind = L.kind;
                U.elem_start = L.elem_start;
                U.elem_end = L.elem_end;
                U.n_af = L.n_af;
                U.feat_tab = L.feat_tab;
                U.af_tab = L.af_tab;
                U.norm_off = L.norm_off;
                U.alpha = L.alpha;
                U.beta = L.beta;
                U.ldj_const = L.ldj_const;
                if (L.kind != DF_LAYER_NORM) {
                    bool ok = make_unet(L.t_dense0, L.t_ndense, &U.t);
                    if (L.kind == DF_LAYER_RNVP) ok = ok && make_unet(L.s_dense0, L.s_ndense, &U.s);
                    if (!ok) fail(DF_ERR_UNSUPPORTED, "internal: default-shape net with an irregular layout");
                    U.s.fold0 = U.t.fold0 = fold[P.ulayers.size()];
                }
                P.ulayers.push_back(U);
            }
            if (!P.uniform) P.ulayers.clear();
        }

        const int nbuf = P.stages.size() > 1 ? 2 : 1;
        const int fixed = nbuf * P.stage_max + table_lds_bytes(P);
        const int per_tile = kWavesPerBlock * 16 * P.stride * 4;
        P.tiles = 1;
        if (resident)
            while (P.tiles < kMaxTilesPerWave && fixed + (P.tiles + 1) * per_tile <= kLdsPerBlockTarget) ++P.tiles;
        if (P.uniform) {  // the specialised kernel evaluates tiles in groups
            P.tile_group = P.fast ? kFastTileGroup : kUniformTileGroup;
            if (P.fast && P.tiles < P.tile_group) {  // not enough LDS for a FAST tile group
                P.fast = 0;
                P.tile_group = kUniformTileGroup;
            }
            if (P.tiles < P.tile_group) fail(DF_ERR_UNSUPPORTED, "LDS too small for the specialised kernel");
            P.tiles -= P.tiles % P.tile_group;
        }
        P.samples_per_block = kWavesPerBlock * 16 * P.tiles;
        if (table_lds_ints(P) > kMaxTableInts)
            fail(DF_ERR_UNSUPPORTED, params_in_lds(P) ? "chain index tables and NormalizationLayer bounds exceed 16 KiB"
                                                      : "chain index tables exceed 16 KiB");
        if (P.stages.empty()) {  // normalization-only chain: keep one empty stage record
            P.stage_max = 0;
        }
        P.blob.resize(round_up((int)P.blob.size(), 16) + 16, 0);
        if (exact < 0) {
            const char* e = std::getenv("DF_F32_EXACT");
            exact = (e && e[0] == '1') ? 1 : 0;
        }
        if (!exact) build_split(desc, P, fold);
        build_wide(desc, P);
        if (!exact) build_wide_split(desc, P);
        *out = std::move(P);
        return DF_OK;
    } catch (const Fail& f) {
        if (err) *err = f.msg;
        return f.code;
    } catch (const std::exception& e) {
        if (err) *err = e.what();
        return DF_ERR_INVALID;
    }
}

}  // namespace df
