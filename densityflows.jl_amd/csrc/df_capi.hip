// df_capi.hip — the C ABI declared in include/densityflows_hip.h.
//
// Host-side only: builds the packed plan (df_plan.cpp), owns the device copy
// of it, and launches the fused kernels (df_kernels_ht*.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "densityflows_hip.h"
#include "df_kernels.h"
#include "df_plan.h"

#include "df_handle.h"

namespace df {
namespace api {

namespace {
thread_local std::string g_err;
}

int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_err(hipError_t e, const char* where) {
    return set_err(DF_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

const char* last_error() { return g_err.c_str(); }

}  // namespace api
}  // namespace df

using namespace df::api;

static size_t lds_for_tiles(const df_chain* c, int t, bool split);

static int uniform_variant(const df::Plan& P, bool split = false) {
    return P.uniform ? (P.fast ? (split ? 4 : 3) : P.relu_only ? 2 : 1) : 0;
}

// The SPLIT blobs exist only when the chain was planned without DF_F32_EXACT=1
// (build_split / build_wide_split read it once, at df_chain_create).
bool use_split(const df_chain* c) { return c->plan.split && !c->exact; }

bool use_wsplit(const df_chain* c) { return c->plan.wsplit && !c->exact; }

// The descriptor of the small-batch kernel (df_kernels.h SmallDesc) for this launch.
static df::SmallDesc small_desc(const df_chain* c, bool flow) {
    const df::Plan& P = c->plan;
    df::SmallDesc sd{};
    for (int li = 0; li < P.n_layers && li < df::kSmallLayers; ++li) {
        const df::ULayer& U = P.ulayers[li];
        sd.kind[li] = (int8_t)U.kind;
        sd.elem_start[li] = (int8_t)U.elem_start;
        sd.elem_end[li] = (int8_t)U.elem_end;
        sd.alpha[li] = U.alpha;
        sd.beta[li] = U.beta;
        sd.ldj_const[li] = U.ldj_const;
        if (U.kind == DF_LAYER_NORM) {
            for (int i = 0; i < P.d && i < 8; ++i) {
                sd.xmin[li][i] = P.params[U.norm_off + i];
                sd.xmax[li][i] = P.params[U.norm_off + P.d + i];
            }
            continue;
        }
        sd.n_out[li] = (int8_t)U.t.n_out;
        for (int k = 0; k < 4; ++k) {
            sd.feat[li][k] = (int8_t)P.tables[U.feat_tab + k];
            sd.af[li][k] = (int8_t)(k < U.n_af ? P.tables[U.af_tab + k] : 0);
        }
        const df::UNet* nets[2] = {&U.s, &U.t};
        for (int k = 0; k < 2; ++k) {
            if (k == 0 && U.kind != DF_LAYER_RNVP) continue;
            const int64_t base = P.stages[nets[k]->stage].src_off;
            sd.w0[li][k] = (int32_t)(base + nets[k]->off_w0);
            sd.wh[li][k] = (int32_t)(base + nets[k]->off_h);
            sd.wo[li][k] = (int32_t)(base + nets[k]->off_out);
        }
    }
    (void)flow;
    return sd;
}

// The small-batch kernel (df_small.hip) for a batch that underfills the chip: FAST
// exact-f32 chains (relu _dflt_net, one hidden Dense, folded first-Dense bias, <= 4
// outputs) of hidden 16 with n + d <= 8 and at most 4 layers (the README chain of
// config 1).  DF_SMALL_MAX (samples) moves the crossover; 0 disables it.
static bool use_small(const df_chain* c, int64_t batch) {
    const df::Plan& P = c->plan;
    if (!(P.uniform && P.fast && P.outv && P.ht == 1 && P.n + P.d <= 8 && P.n_layers <= df::kSmallLayers))
        return false;
    const int64_t max_b = c->small_max >= 0 ? c->small_max : (int64_t)df::kSmallSamples * 8 * c->n_cu;
    return batch <= max_b;
}

static size_t lds_for_tiles(const df_chain* c, int t, bool split = false) {
    const df::Plan& P = c->plan;
    if (split)
        return (size_t)c->sstage_bytes * c->sn_stage_bufs + c->tab_bytes +
               (size_t)df::kWavesPerBlock * 16 * t * P.stride * 4;
    return (size_t)c->stage_bytes * c->n_stage_bufs + c->tab_bytes +
           (size_t)df::kWavesPerBlock * 16 * t * P.stride * 4;
}

// Tiles per wave for this launch: balance the grid over the resident
// workgroup slots (time ~ rounds × (tiles + fixed per-round overhead)).
static int choose_tiles(const df_chain* c, int mode, int64_t batch, bool split) {
    const df::Plan& P = c->plan;
    const int max_t = split ? P.stiles : P.tiles;
    const int (*occ)[df::kMaxTilesPerWave + 1] = split ? c->socc : c->occ;
    if (c->force_tiles > 0) {  // tuning knob (DF_TILES): force the tiles per wave
        const int t = c->force_tiles;
        const int step = P.uniform ? P.tile_group : 1;
        if (t >= 1 && t <= max_t && t % step == 0) return t;
    }
    int best = P.uniform ? P.tile_group : 1;
    double best_cost = 1e300;
    const int step = P.uniform ? P.tile_group : 1;
    for (int t = step; t <= max_t; t += step) {
        const int64_t per_block = (int64_t)df::kWavesPerBlock * 16 * t;
        const int64_t nwg = (batch + per_block - 1) / per_block;
        const int64_t slots = (int64_t)c->n_cu * (occ[mode][t] > 0 ? occ[mode][t] : 1);
        const int64_t rounds = (nwg + slots - 1) / slots;
        const double cost = (double)rounds * (t + 0.5);
        if (cost <= best_cost) {
            best_cost = cost;
            best = t;
        }
    }
    return best;
}

template <typename T>
static bool same_bytes(const std::vector<T>& a, const std::vector<T>& b) {
    return a.size() == b.size() && (a.empty() || std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0);
}

template <typename T>
static int refresh(const std::vector<T>& v, void* dst) {
    if (v.empty()) return DF_OK;
    hipError_t e = hipMemcpy(dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
    return e == hipSuccess ? DF_OK : hip_err(e, "hipMemcpy(weights)");
}

extern "C" {

int df_get_abi_version(void) { return DF_ABI_VERSION; }

const char* df_last_error(void) { return last_error(); }

int df_get_limits(df_limits* out) {
    if (!out) return set_err(DF_ERR_INVALID, "null pointer");
    out->max_state = df::kMaxState;
    out->max_hidden = df::kMaxHidden;
    out->max_af = df::kMaxAf;
    out->max_layers = df::kMaxLayers;
    return DF_OK;
}

int df_chain_destroy(df_chain* c) {
    if (!c) return DF_OK;
    if (c->n_trainers > 0) return set_err(DF_ERR_INVALID, "df_chain_destroy: destroy its df_train handles first");
    DeviceGuard gd(c->device);
    void* ptrs[] = {c->d_layers, c->d_denses, c->d_chunks,  c->d_stages,  c->d_blob,  c->d_tables,
                    c->d_params, c->d_bounds, c->d_partial, c->d_sched,   c->d_ulayers, c->d_wlayers,
                    c->d_wstages, c->d_wblob, c->d_wbias,  c->d_wsched, c->d_sblob, c->d_sstages,
                    c->d_ssched,  c->d_sulayers, c->d_wslayers, c->d_wsstages, c->d_wsblob, c->d_wssched,
                    c->d_wstables, c->d_clk, c->d_theta_ws};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete c;
    return DF_OK;
}

int df_chain_create(df_chain** out, const df_chain_desc* desc, int device) {
    if (!out) return set_err(DF_ERR_INVALID, "null output handle");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return set_err(DF_ERR_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return set_err(DF_ERR_INVALID, "device ordinal out of range");
    df_chain* c = new (std::nothrow) df_chain();
    if (!c) return set_err(DF_ERR_NOMEM, "host allocation failed");
    std::string err;
    const char* ex = std::getenv("DF_F32_EXACT");   // the chain's arithmetic, read once
    c->exact = ex && ex[0] == '1';
    c->no_wide = std::getenv("DF_NO_WIDE") && std::getenv("DF_NO_WIDE")[0] == '1';
    c->debug_launch = std::getenv("DF_DEBUG_LAUNCH") && std::getenv("DF_DEBUG_LAUNCH")[0] == '1';
    if (const char* e = std::getenv("DF_TILES")) c->force_tiles = std::atoi(e);
    if (const char* e = std::getenv("DF_SMALL_MAX")) c->small_max = std::max<int64_t>(0, std::atoll(e));
    if (const char* e = std::getenv("DF_SMALL_WAVES")) c->small_waves = std::atoi(e) == 1 ? 1 : 2;
    int rc = df::build_plan(desc, &c->plan, &err, c->exact ? 1 : 0);
    if (rc != DF_OK) {
        delete c;
        return set_err(rc, err);
    }
    c->device = device;
    DeviceGuard gd(device);
    if (!gd.ok) {
        delete c;
        return set_err(DF_ERR_HIP, "hipSetDevice failed");
    }
    const df::Plan& P = c->plan;
    std::vector<int32_t> sched_all(P.sched_fwd);
    sched_all.insert(sched_all.end(), P.sched_bwd.begin(), P.sched_bwd.end());
    if ((rc = upload(P.layers, &c->d_layers)) != DF_OK || (rc = upload(P.denses, &c->d_denses)) != DF_OK ||
        (rc = upload(P.chunks, &c->d_chunks)) != DF_OK || (rc = upload(P.stages, &c->d_stages)) != DF_OK ||
        (rc = upload(P.blob, &c->d_blob)) != DF_OK || (rc = upload(P.tables, &c->d_tables)) != DF_OK ||
        (rc = upload(P.params, &c->d_params)) != DF_OK || (rc = upload(sched_all, &c->d_sched)) != DF_OK ||
        (rc = upload(P.ulayers, &c->d_ulayers)) != DF_OK) {
        std::string m = g_err;
        df_chain_destroy(c);
        return set_err(rc, m);
    }
    if (P.wide) {
        std::vector<int32_t> wsched(P.wsched_fwd);
        wsched.insert(wsched.end(), P.wsched_bwd.begin(), P.wsched_bwd.end());
        if ((rc = upload(P.wlayers, &c->d_wlayers)) != DF_OK || (rc = upload(P.wstages, &c->d_wstages)) != DF_OK ||
            (rc = upload(P.wblob, &c->d_wblob)) != DF_OK || (rc = upload(P.wbias, &c->d_wbias)) != DF_OK ||
            (rc = upload(wsched, &c->d_wsched)) != DF_OK) {
            std::string m = last_error();
            df_chain_destroy(c);
            return set_err(rc, m);
        }
    }
    if (P.split) {
        std::vector<int32_t> ssched(P.ssched_fwd);
        ssched.insert(ssched.end(), P.ssched_bwd.begin(), P.ssched_bwd.end());
        if ((rc = upload(P.sulayers, &c->d_sulayers)) != DF_OK || (rc = upload(P.sstages, &c->d_sstages)) != DF_OK ||
            (rc = upload(P.sblob, &c->d_sblob)) != DF_OK || (rc = upload(ssched, &c->d_ssched)) != DF_OK) {
            std::string m = last_error();
            df_chain_destroy(c);
            return set_err(rc, m);
        }
    }
    if (P.wsplit) {
        std::vector<int32_t> wssched(P.wssched_fwd);
        wssched.insert(wssched.end(), P.wssched_bwd.begin(), P.wssched_bwd.end());
        if ((rc = upload(P.wslayers, &c->d_wslayers)) != DF_OK || (rc = upload(P.wsstages, &c->d_wsstages)) != DF_OK ||
            (rc = upload(P.wsblob, &c->d_wsblob)) != DF_OK || (rc = upload(wssched, &c->d_wssched)) != DF_OK ||
            (rc = upload(P.wstables, &c->d_wstables)) != DF_OK) {
            std::string m = last_error();
            df_chain_destroy(c);
            return set_err(rc, m);
        }
    }
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->d_bounds), sizeof(float) * (2 * P.n + 4));
    if (e != hipSuccess) {
        df_chain_destroy(c);
        return set_err(DF_ERR_NOMEM, "hipMalloc failed (θ bounds)");
    }
    // LDS carve: [stage buffer(s) | tables | state tile]; the stage area also hosts
    // the fp64 workgroup reduction of the logpdf epilogue (>= 64 B).
    c->stage_bytes = P.stage_max < 1024 ? 1024 : P.stage_max;
    c->n_stage_bufs = P.stages.size() > 1 ? 2 : 1;
    c->tab_bytes = df::table_lds_bytes(P);
    c->lds = (size_t)c->stage_bytes * c->n_stage_bufs + c->tab_bytes +
             (size_t)P.samples_per_block * P.stride * 4;
    if (c->lds > 160 * 1024) {
        df_chain_destroy(c);
        return set_err(DF_ERR_UNSUPPORTED, "chain needs more than 160 KiB of LDS per workgroup");
    }
    if (P.wide) {
        c->wide_lds = (size_t)df::kWideBufs * df::kWideStageBytes + c->tab_bytes +
                      (size_t)df::kWideWaves * 16 * df::kWideT * P.stride * 4;
        e = df::set_wide_lds_limit(c->wide_lds);
        if (e != hipSuccess) {
            df_chain_destroy(c);
            return hip_err(e, "hipFuncSetAttribute(wide)");
        }
        if (P.wsplit) {
            c->wstab_bytes = ((int)P.wstables.size() * 4 + 15) / 16 * 16;
            c->wslds = (size_t)df::kWideSplitBufs * df::kWideSplitStageBytes + c->wstab_bytes +
                       (size_t)df::kWideWaves * 16 * df::kWideT * P.stride * 4;
            if (c->wslds > 160 * 1024) {
                df_chain_destroy(c);
                return set_err(DF_ERR_UNSUPPORTED, "wide SPLIT kernel needs more than 160 KiB of LDS");
            }
            e = df::set_wide_lds_limit(c->wslds, true);
            if (e != hipSuccess) {
                df_chain_destroy(c);
                return hip_err(e, "hipFuncSetAttribute(wide split)");
            }
        }
    }
    if (P.split) {
        c->sstage_bytes = P.sstage_max;
        c->sn_stage_bufs = P.sstages.size() > 1 ? 2 : 1;
        c->slds = lds_for_tiles(c, P.stiles, true);
    }
    e = df::set_kernel_lds_limit(P.ht, P.uniform != 0, std::max(c->lds, c->slds));
    if (e != hipSuccess) {
        df_chain_destroy(c);
        return hip_err(e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
    }
    // occupancy by mode and tiles per wave (for the per-launch tile choice)
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->n_cu < 1)
        c->n_cu = 256;
    for (int mode = 0; mode < 4; ++mode)
        for (int t = 1; t <= P.tiles; ++t) {
            int blocks = 1;
            if (df::kernel_occupancy(P.ht, mode, P.outv != 0, uniform_variant(P), lds_for_tiles(c, t, false),
                                     &blocks) != hipSuccess ||
                blocks < 1)
                blocks = 1;
            c->occ[mode][t] = blocks;
        }
    for (int mode = 0; mode < 4 && P.split; ++mode)
        for (int t = 1; t <= P.stiles; ++t) {
            int blocks = 1;
            if (df::kernel_occupancy(P.ht, mode, true, 4, lds_for_tiles(c, t, true), &blocks) != hipSuccess ||
                blocks < 1)
                blocks = 1;
            c->socc[mode][t] = blocks;
        }
    *out = c;
    return DF_OK;
}

static void fill_info(const df::Plan& P, df_chain_info* out) {
    out->d = P.d;
    out->n = P.n;
    out->n_layers = P.n_layers;
    out->hidden_tiles = P.ht;
    out->samples_per_block = P.samples_per_block;
    out->n_stages = (int32_t)P.stages.size();
    out->n_params = P.n_params;
    out->flops_per_sample = P.flops_per_sample;
    out->weight_bytes = (int64_t)P.blob.size();
    out->kernel = P.wide ? (P.wsplit ? 6 : 5) : P.split ? 4 : uniform_variant(P);
    out->reserved = 0;
    out->split_flops_per_sample = (P.split || P.wsplit) ? P.split_flops_per_sample : 0.0;
}

int df_chain_get_info(const df_chain* c, df_chain_info* out) {
    if (!c || !out) return set_err(DF_ERR_INVALID, "null pointer");
    fill_info(c->plan, out);
    return DF_OK;
}

int df_chain_validate(const df_chain_desc* desc, df_chain_info* info) {
    df::Plan P;
    std::string err;
    int rc = df::build_plan(desc, &P, &err);
    if (rc != DF_OK) return set_err(rc, err);
    if (info) fill_info(P, info);
    return DF_OK;
}

int df_chain_set_weights(df_chain* c, const df_chain_desc* desc) {
    if (!c || !desc) return set_err(DF_ERR_INVALID, "null pointer");
    if (c->n_trainers > 0)
        return set_err(DF_ERR_INVALID, "df_chain_set_weights: a df_train handle owns the parameters "
                                       "(use df_train_set_params)");
    df::Plan P;
    std::string err;
    int rc = df::build_plan(desc, &P, &err, c->exact ? 1 : 0);   // the chain's arithmetic, not today's env
    if (rc != DF_OK) return set_err(rc, err);
    const df::Plan& Q = c->plan;
    // structure: everything but the parameter values (and the ldj constants of the
    // NormalizationLayers, which follow from x_min / x_max) must be identical
    const bool same = P.d == Q.d && P.n == Q.n && P.n_layers == Q.n_layers && P.ht == Q.ht && P.tiles == Q.tiles &&
                      P.outv == Q.outv && P.uniform == Q.uniform && P.relu_only == Q.relu_only && P.fast == Q.fast &&
                      P.wide == Q.wide && P.stride == Q.stride && P.layers.size() == Q.layers.size() &&
                      same_bytes(P.denses, Q.denses) && same_bytes(P.chunks, Q.chunks) &&
                      same_bytes(P.stages, Q.stages) && same_bytes(P.tables, Q.tables) &&
                      same_bytes(P.sched_fwd, Q.sched_fwd) && same_bytes(P.sched_bwd, Q.sched_bwd) &&
                      P.blob.size() == Q.blob.size() && P.params.size() == Q.params.size() &&
                      P.ulayers.size() == Q.ulayers.size() && P.wlayers.size() == Q.wlayers.size() &&
                      same_bytes(P.wstages, Q.wstages) && P.wblob.size() == Q.wblob.size() &&
                      P.wbias.size() == Q.wbias.size() && same_bytes(P.pack_dst, Q.pack_dst) &&
                      P.split == Q.split && same_bytes(P.sstages, Q.sstages) && P.sblob.size() == Q.sblob.size() &&
                      P.wsplit == Q.wsplit && same_bytes(P.wsstages, Q.wsstages) && P.wsblob.size() == Q.wsblob.size();
    if (!same) return set_err(DF_ERR_SHAPE, "df_chain_set_weights: the descriptor's structure differs from the chain's");
    for (size_t i = 0; i < P.layers.size(); ++i)
        if (P.layers[i].kind != Q.layers[i].kind || P.layers[i].n_af != Q.layers[i].n_af)
            return set_err(DF_ERR_SHAPE, "df_chain_set_weights: layer structure differs");
    DeviceGuard gd(c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    hipError_t e = hipDeviceSynchronize();  // no launch may still read the old weights
    if (e != hipSuccess) return hip_err(e, "hipDeviceSynchronize");
    if ((rc = refresh(P.layers, c->d_layers)) != DF_OK || (rc = refresh(P.blob, c->d_blob)) != DF_OK ||
        (rc = refresh(P.params, c->d_params)) != DF_OK || (rc = refresh(P.ulayers, c->d_ulayers)) != DF_OK)
        return rc;
    if (P.wide && ((rc = refresh(P.wlayers, c->d_wlayers)) != DF_OK || (rc = refresh(P.wblob, c->d_wblob)) != DF_OK ||
                   (rc = refresh(P.wbias, c->d_wbias)) != DF_OK))
        return rc;
    if (P.split && ((rc = refresh(P.sulayers, c->d_sulayers)) != DF_OK || (rc = refresh(P.sblob, c->d_sblob)) != DF_OK))
        return rc;
    if (P.wsplit && ((rc = refresh(P.wslayers, c->d_wslayers)) != DF_OK || (rc = refresh(P.wsblob, c->d_wsblob)) != DF_OK))
        return rc;
    c->plan.layers = P.layers;
    c->plan.ulayers = P.ulayers;
    c->plan.wlayers = P.wlayers;
    c->plan.blob.swap(P.blob);
    c->plan.params.swap(P.params);
    c->plan.wblob.swap(P.wblob);
    c->plan.wbias.swap(P.wbias);
    c->plan.sulayers = P.sulayers;
    c->plan.sblob.swap(P.sblob);
    c->plan.wslayers = P.wslayers;
    c->plan.wsblob.swap(P.wsblob);
    c->plan.trainables.swap(P.trainables);
    c->small_sd_ok[0] = c->small_sd_ok[1] = false;
    return DF_OK;
}

int df_chain_set_theta_bounds(df_chain* c, const float* tmin, const float* tmax) {
    if (!c) return set_err(DF_ERR_INVALID, "null chain");
    const int n = c->plan.n;
    if (n == 0) {
        c->has_bounds = false;
        return DF_OK;
    }
    if (!tmin || !tmax) return set_err(DF_ERR_INVALID, "null θ bounds");
    std::vector<float> b(2 * n);
    std::memcpy(b.data(), tmin, sizeof(float) * n);
    std::memcpy(b.data() + n, tmax, sizeof(float) * n);
    DeviceGuard gd(c->device);
    hipError_t e = hipMemcpy(c->d_bounds, b.data(), sizeof(float) * 2 * n, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_err(e, "hipMemcpy(θ bounds)");
    c->h_bounds = b;
    c->has_bounds = true;
    c->small_sd_ok[1] = false;
    return DF_OK;
}

}  // extern "C"

namespace df {
namespace api {

int run(df_chain* c, int mode, bool flow, const float* zin, const float* theta, float* xout, float* ldj, float* lp,
        double* sum_out, int64_t batch, void* stream, float* snap, float* hsave, int hsave_w, int hsave_h,
        float* fsave) {
    if (!c) return set_err(DF_ERR_INVALID, "null chain");
    if (batch < 0) return set_err(DF_ERR_SHAPE, "negative batch size");
    const df::Plan& P = c->plan;
    if (batch == 0) {
        if (sum_out) {
            DeviceGuard gd(c->device);
            hipError_t e = hipMemsetAsync(sum_out, 0, sizeof(double), (hipStream_t)stream);
            if (e != hipSuccess) return hip_err(e, "hipMemsetAsync");
        }
        return DF_OK;
    }
    if (!zin) return set_err(DF_ERR_INVALID, "null input array");
    if (P.n > 0 && !theta)
        return set_err(DF_ERR_SHAPE, "dimensions θ must match (n, dims...) with n number of trained parameters");
    if (mode != df::MODE_LOGPDF && !xout) return set_err(DF_ERR_INVALID, "null output array");
    if (flow && P.n > 0 && !c->has_bounds) return set_err(DF_ERR_INVALID, "θ bounds not set (df_chain_set_theta_bounds)");

    DeviceGuard gd(c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    const bool wide = P.wide && !c->no_wide;
    const bool split = !wide && use_split(c);
    const bool small = !wide && !split && use_small(c, batch);
    if (fsave && !(wide && use_wsplit(c)))  // the trainer plans its H0-free sweep on the wide SPLIT kernel
        return set_err(DF_ERR_INVALID, "internal: feature snapshots need the wide SPLIT kernel");
    // (the small kernel runs one 16-sample tile per workgroup: tiles = 1, only reported)
    const int tiles = wide ? df::kWideT : small ? 1 : choose_tiles(c, mode, batch, split);
    {
        if (c->debug_launch) {  // tuning aid (DF_DEBUG_LAUNCH=1): the launch shape on stderr
            std::fprintf(stderr, "[df] mode %d batch %lld kernel %s tiles %d (max %d) occupancy:", mode,
                         (long long)batch,
                         wide ? (use_wsplit(c) ? "wide-split" : "wide") : small ? "small" : !P.uniform ? "generic" : split ? "uniform-fast-split" : P.fast ? "uniform-fast" : "uniform",
                         tiles, split ? P.stiles : P.tiles);
            for (int t = 1; t <= (split ? P.stiles : P.tiles); ++t)
                std::fprintf(stderr, " t%d=%d", t, split ? c->socc[mode][t] : c->occ[mode][t]);
            std::fprintf(stderr, "\n");
        }
    }
    const int64_t S = wide ? (int64_t)df::kWideWaves * 16 * df::kWideT
                           : small ? (int64_t)df::kSmallSamples : (int64_t)df::kWavesPerBlock * 16 * tiles;
    const int64_t grid = (batch + S - 1) / S;
    if (grid > 0x7fffffff) return set_err(DF_ERR_UNSUPPORTED, "batch too large for one launch");
    if (sum_out && grid > c->partial_cap) {
        if (c->d_partial) (void)hipFree(c->d_partial);
        c->d_partial = nullptr;
        c->partial_cap = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->d_partial), sizeof(double) * grid);
        if (e != hipSuccess) return set_err(DF_ERR_NOMEM, "hipMalloc failed (NLL partials)");
        c->partial_cap = grid;
        c->partial_gen++;
    }

    // Clock stamps are an eager-launch diagnostic: a launch recorded into a stream
    // capture (df_train_step_graph) never stamps, so no graph names d_clk and no
    // allocation runs inside a capture.
    hipStreamCaptureStatus cap_status = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cap_status) != hipSuccess) cap_status = hipStreamCaptureStatusNone;
    const bool stamp = c->clk_on && cap_status == hipStreamCaptureStatusNone;
    if (stamp && grid > c->clk_cap) {  // stamp slots for this grid (zeroed: a new series)
        if (c->d_clk) (void)hipFree(c->d_clk);
        c->d_clk = nullptr;
        c->clk_cap = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->d_clk), sizeof(uint64_t) * 2 * grid);
        if (e == hipSuccess) e = hipMemsetAsync(c->d_clk, 0, sizeof(uint64_t) * 2 * grid, (hipStream_t)stream);
        if (e != hipSuccess) return set_err(DF_ERR_NOMEM, "hipMalloc failed (clock stamps)");
        c->clk_cap = grid;
    }

    df::ChainArgs a{};
    a.clk = stamp ? c->d_clk : nullptr;
    a.zin = zin;
    a.theta = theta;
    a.xout = xout;
    a.ldj_out = ldj;
    a.lp_out = lp;
    a.partial = sum_out ? c->d_partial : nullptr;
    a.batch = batch;
    a.layers = static_cast<const df::DevLayer*>(c->d_layers);
    a.denses = static_cast<const df::DevDense*>(c->d_denses);
    a.chunks = static_cast<const df::DevChunk*>(c->d_chunks);
    a.stages = static_cast<const df::DevStage*>(c->d_stages);
    a.blob = static_cast<const uint8_t*>(c->d_blob);
    a.tables = static_cast<const int32_t*>(c->d_tables);
    a.params = static_cast<const float*>(c->d_params);
    a.tmin = (flow && P.n > 0) ? c->d_bounds : nullptr;
    a.tmax = (flow && P.n > 0) ? c->d_bounds + P.n : nullptr;
    a.d = P.d;
    a.n = P.n;
    a.stride = P.stride;
    a.tiles = tiles;
    a.ulayers = static_cast<const df::ULayer*>(c->d_ulayers);
    a.n_layers = P.n_layers;
    a.tab_ints = (int)P.tables.size();
    a.tab_bytes = c->tab_bytes;
    a.n_par = (int)P.params.size();
    a.stage_bytes = c->stage_bytes;
    a.n_stage_bufs = c->n_stage_bufs;
    a.sched_fwd = static_cast<const int32_t*>(c->d_sched);
    a.sched_bwd = a.sched_fwd + P.sched_fwd.size();
    a.n_sched_fwd = (int)P.sched_fwd.size();
    a.n_sched_bwd = (int)P.sched_bwd.size();
    // Distributions.mvnormal_c0: -(d * log2π + logdetcov)/2 in Float32, logdet(I) = 0
    a.c0 = -((float)P.d * (float)kLog2Pi + 0.f) / 2.f;
    a.snap = snap;
    a.hsave = P.uniform ? nullptr : hsave;
    a.hsave_w = hsave_w;
    a.hsave_h = hsave_h;
    a.fsave = nullptr;

    hipStream_t st = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (wide) {
        a.blob = static_cast<const uint8_t*>(c->d_wblob);
        a.stages = static_cast<const df::DevStage*>(c->d_wstages);
        a.sched_fwd = static_cast<const int32_t*>(c->d_wsched);
        a.sched_bwd = a.sched_fwd + P.wsched_fwd.size();
        a.n_sched_fwd = (int)P.wsched_fwd.size();
        a.n_sched_bwd = (int)P.wsched_bwd.size();
        a.wlayers = static_cast<const df::WLayer*>(c->d_wlayers);
        a.wbias = static_cast<const float*>(c->d_wbias);
        if (use_wsplit(c)) {
            a.blob = static_cast<const uint8_t*>(c->d_wsblob);
            a.stages = static_cast<const df::DevStage*>(c->d_wsstages);
            a.sched_fwd = static_cast<const int32_t*>(c->d_wssched);
            a.sched_bwd = a.sched_fwd + P.wssched_fwd.size();
            a.n_sched_fwd = (int)P.wssched_fwd.size();
            a.n_sched_bwd = (int)P.wssched_bwd.size();
            a.wlayers = static_cast<const df::WLayer*>(c->d_wslayers);
            a.tables = static_cast<const int32_t*>(c->d_wstables);
            a.tab_ints = (int)P.wstables.size();
            a.tab_bytes = c->wstab_bytes;
            a.fsave = fsave;  // features instead of H0 (the split kernel only)
            e = df::launch_wide(mode, a, (unsigned)grid, c->wslds, st, true);
        } else {
            e = df::launch_wide(mode, a, (unsigned)grid, c->wide_lds, st);
        }
    } else if (small) {
        const int fi = flow ? 1 : 0;
        if (!c->small_sd_ok[fi]) {
            c->small_sd[fi] = small_desc(c, flow);
            c->small_sd_ok[fi] = true;
        }
        e = df::launch_small(mode, a, c->small_sd[fi], (unsigned)grid, st, c->small_waves);
    } else if (split) {
        a.blob = static_cast<const uint8_t*>(c->d_sblob);
        a.stages = static_cast<const df::DevStage*>(c->d_sstages);
        a.ulayers = static_cast<const df::ULayer*>(c->d_sulayers);
        a.stage_bytes = c->sstage_bytes;
        a.n_stage_bufs = c->sn_stage_bufs;
        a.sched_fwd = static_cast<const int32_t*>(c->d_ssched);
        a.sched_bwd = a.sched_fwd + P.ssched_fwd.size();
        a.n_sched_fwd = (int)P.ssched_fwd.size();
        a.n_sched_bwd = (int)P.ssched_bwd.size();
        e = df::launch_chain(P.ht, mode, true, 4, a, (unsigned)grid, lds_for_tiles(c, tiles, true), st);
    } else {
        e = df::launch_chain(P.ht, mode, P.outv != 0, uniform_variant(P), a, (unsigned)grid,
                             lds_for_tiles(c, tiles, false), st);
    }
    if (e != hipSuccess) return hip_err(e, "chain kernel launch");
    if (sum_out) {
        e = df::launch_reduce_partials(c->d_partial, grid, sum_out, st);
        if (e != hipSuccess) return hip_err(e, "reduce kernel launch");
    }
    return DF_OK;
}

}  // namespace api
}  // namespace df

extern "C" {

int df_chain_forward(df_chain* c, const float* z, const float* theta, float* x_out, float* ldj_out, int64_t batch,
                     void* stream) {
    return run(c, df::MODE_FWD, false, z, theta, x_out, ldj_out, nullptr, nullptr, batch, stream);
}

int df_chain_backward(df_chain* c, const float* x, const float* theta, float* z_out, float* ldj_out, int64_t batch,
                      void* stream) {
    return run(c, df::MODE_BWD, false, x, theta, z_out, ldj_out, nullptr, nullptr, batch, stream);
}

int df_chain_forward_inplace(df_chain* c, float* z, const float* theta, int64_t batch, void* stream) {
    return run(c, df::MODE_FWD_INPLACE, false, z, theta, z, nullptr, nullptr, nullptr, batch, stream);
}

int df_flow_forward(df_chain* c, const float* z, const float* theta_raw, float* x_out, float* ldj_out,
                    int64_t batch, void* stream) {
    return run(c, df::MODE_FWD, true, z, theta_raw, x_out, ldj_out, nullptr, nullptr, batch, stream);
}

int df_flow_backward(df_chain* c, const float* x, const float* theta_raw, float* z_out, float* ldj_out,
                     int64_t batch, void* stream) {
    return run(c, df::MODE_BWD, true, x, theta_raw, z_out, ldj_out, nullptr, nullptr, batch, stream);
}

int df_flow_forward_inplace(df_chain* c, float* z, const float* theta_raw, int64_t batch, void* stream) {
    return run(c, df::MODE_FWD_INPLACE, true, z, theta_raw, z, nullptr, nullptr, nullptr, batch, stream);
}

int df_flow_logpdf(df_chain* c, const float* x, const float* theta_raw, float* logpdf_out, int64_t batch,
                   void* stream) {
    if (batch > 0 && !logpdf_out) return set_err(DF_ERR_INVALID, "null logpdf output");
    return run(c, df::MODE_LOGPDF, true, x, theta_raw, nullptr, nullptr, logpdf_out, nullptr, batch, stream);
}

int df_flow_logpdf_sum(df_chain* c, const float* x, const float* theta_raw, double* sum_out, int64_t batch,
                       void* stream) {
    if (!sum_out) return set_err(DF_ERR_INVALID, "null sum output");
    return run(c, df::MODE_LOGPDF, true, x, theta_raw, nullptr, nullptr, nullptr, sum_out, batch, stream);
}

int df_chain_logpdf(df_chain* c, const float* x, const float* theta, float* logpdf_out, int64_t batch,
                    void* stream) {
    if (batch > 0 && !logpdf_out) return set_err(DF_ERR_INVALID, "null logpdf output");
    return run(c, df::MODE_LOGPDF, false, x, theta, nullptr, nullptr, logpdf_out, nullptr, batch, stream);
}

int df_chain_logpdf_sum(df_chain* c, const float* x, const float* theta, double* sum_out, int64_t batch,
                        void* stream) {
    if (!sum_out) return set_err(DF_ERR_INVALID, "null sum output");
    return run(c, df::MODE_LOGPDF, false, x, theta, nullptr, nullptr, nullptr, sum_out, batch, stream);
}

int df_chain_clock_probe(df_chain* c, int on) {
    if (!c) return set_err(DF_ERR_INVALID, "null chain");
    DeviceGuard gd(c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    if (on && c->d_clk) {
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess) e = hipMemset(c->d_clk, 0, sizeof(uint64_t) * 2 * c->clk_cap);
        if (e != hipSuccess) return hip_err(e, "hipMemset(clock stamps)");
    }
    c->clk_on = on != 0;
    return DF_OK;
}

int df_chain_clock_read(df_chain* c, double* ghz_median, double* ghz_mean, int64_t* n_slots) {
    if (!c || !ghz_median || !ghz_mean || !n_slots) return set_err(DF_ERR_INVALID, "null pointer");
    *ghz_median = *ghz_mean = 0.0;
    *n_slots = 0;
    if (!c->d_clk || c->clk_cap == 0) return DF_OK;
    DeviceGuard gd(c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    std::vector<uint64_t> h((size_t)2 * c->clk_cap);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h.data(), c->d_clk, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_err(e, "hipMemcpy(clock stamps)");
    std::vector<double> ghz;
    double st = 0.0, sr = 0.0;
    for (int64_t b = 0; b < c->clk_cap; ++b) {
        const uint64_t dt = h[2 * b], dr = h[2 * b + 1];
        if (dr == 0) continue;
        ghz.push_back(0.1 * (double)dt / (double)dr);  // s_memrealtime ticks at 100 MHz
        st += (double)dt;
        sr += (double)dr;
    }
    if (ghz.empty()) return DF_OK;
    std::sort(ghz.begin(), ghz.end());
    const size_t m = ghz.size();
    *ghz_median = (m & 1) ? ghz[m / 2] : 0.5 * (ghz[m / 2 - 1] + ghz[m / 2]);
    *ghz_mean = 0.1 * st / sr;
    *n_slots = (int64_t)m;
    return DF_OK;
}

int df_device_alloc(void** ptr, size_t bytes) {
    if (!ptr) return set_err(DF_ERR_INVALID, "null pointer");
    hipError_t e = hipMalloc(ptr, bytes ? bytes : 1);
    return e == hipSuccess ? DF_OK : set_err(DF_ERR_NOMEM, "hipMalloc failed");
}

int df_device_free(void* ptr) {
    hipError_t e = hipFree(ptr);
    return e == hipSuccess ? DF_OK : hip_err(e, "hipFree");
}

int df_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? DF_OK : hip_err(e, "hipMemcpyAsync(H2D)");
}

int df_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? DF_OK : hip_err(e, "hipMemcpyAsync(D2H)");
}

int df_stream_synchronize(void* stream) {
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? DF_OK : hip_err(e, "hipStreamSynchronize");
}

}  // extern "C"
