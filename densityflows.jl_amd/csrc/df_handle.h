// df_handle.h — the df_chain handle and the host helpers shared by the C ABI
// translation units (df_capi.hip: inference entry points, df_train_capi.hip:
// training entry points).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "densityflows_hip.h"
#include "df_kernels.h"
#include "df_plan.h"

struct df_chain {
    df::Plan plan;
    int device = 0;
    bool exact = false;         // DF_F32_EXACT=1 at df_chain_create: exact-f32 kernels only (read once)
    // launch knobs, read from the environment once at df_chain_create (a launch does no
    // getenv): DF_NO_WIDE=1, DF_DEBUG_LAUNCH=1, DF_TILES, DF_SMALL_MAX (-1: unset)
    bool no_wide = false;
    bool debug_launch = false;
    int force_tiles = 0;
    int64_t small_max = -1;
    int small_waves = 2;  // DF_SMALL_WAVES: waves per small-kernel workgroup (1 or 2)
    // the small-batch kernel's descriptor, by flow (θ normalised) 0 / 1; rebuilt after
    // df_chain_set_weights / df_chain_set_theta_bounds
    df::SmallDesc small_sd[2] = {};
    bool small_sd_ok[2] = {false, false};
    void* d_layers = nullptr;
    void* d_denses = nullptr;
    void* d_chunks = nullptr;
    void* d_stages = nullptr;
    void* d_blob = nullptr;
    void* d_tables = nullptr;
    void* d_params = nullptr;
    float* d_bounds = nullptr;  // [θmin (n) | θmax (n)]
    bool has_bounds = false;
    std::vector<float> h_bounds;  // host copy of d_bounds (the small-batch kernel's descriptor)
    double* d_partial = nullptr;
    int64_t partial_cap = 0;
    int64_t partial_gen = 0;  // bumped when d_partial is reallocated (captured train graphs hold it)
    int stage_bytes = 0;
    int n_stage_bufs = 1;
    void* d_sched = nullptr;    // [fwd schedule | bwd schedule]
    void* d_ulayers = nullptr;  // specialised-kernel descriptors
    int n_cu = 0;
    int occ[4][df::kMaxTilesPerWave + 1] = {};  // resident workgroups per CU, by mode and tiles
    int tab_bytes = 0;
    size_t lds = 0;
    int n_trainers = 0;         // live df_train handles bound to this chain
    // wide-net kernel (plan.wide): its own blob, stages, schedules, descriptors
    void* d_wlayers = nullptr;
    void* d_wstages = nullptr;
    void* d_wblob = nullptr;
    void* d_wbias = nullptr;
    void* d_wsched = nullptr;
    size_t wide_lds = 0;
    // SPLIT variant of the FAST kernel (plan.split): its own blob, stages, schedules, descriptors
    void* d_sblob = nullptr;
    void* d_sstages = nullptr;
    void* d_ssched = nullptr;
    void* d_sulayers = nullptr;
    int sstage_bytes = 0;
    int sn_stage_bufs = 1;
    size_t slds = 0;
    int socc[4][df::kMaxTilesPerWave + 1] = {};
    // SPLIT variant of the wide kernel (plan.wsplit)
    void* d_wslayers = nullptr;
    void* d_wsstages = nullptr;
    void* d_wsblob = nullptr;
    void* d_wssched = nullptr;
    void* d_wstables = nullptr;
    int wstab_bytes = 0;
    size_t wslds = 0;
    // effective-clock stamps (df_chain_clock_probe): 2 × uint64 per workgroup slot
    uint64_t* d_clk = nullptr;
    int64_t clk_cap = 0;  // workgroup slots
    bool clk_on = false;
    // θ broadcast workspace of df_flow_sample (NTuple θ)
    float* d_theta_ws = nullptr;
    int64_t theta_ws_cap = 0;
};

// SPLIT launches unless the chain was created under DF_F32_EXACT=1 (df_chain::exact)
bool use_split(const df_chain* c);
bool use_wsplit(const df_chain* c);

namespace df {
namespace api {

int set_err(int code, const std::string& msg);
int hip_err(hipError_t e, const char* where);
const char* last_error();

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && (prev == dev || hipSetDevice(dev) == hipSuccess)) ok = true;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

template <typename T>
int upload(const std::vector<T>& v, void** dst) {
    size_t bytes = v.size() * sizeof(T);
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(dst, bytes);
    if (e != hipSuccess) return set_err(DF_ERR_NOMEM, "hipMalloc failed for the chain plan");
    if (!v.empty()) {
        e = hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_err(e, "hipMemcpy(plan)");
    }
    return DF_OK;
}

constexpr double kLog2Pi = 1.8378770664093453;  // log(2π)

// Device ordinal of a df_train handle (df_train_capi.hip; df_comm.hip checks it).
int train_device(const df_train* t);
// Device double the last df_train_gradient wrote Σ logpdf to (the caller's or the handle's own).
double* train_last_lpsum(df_train* t);

// Launch one fused chain pass.  flow: θ normalised with the handle's bounds;
// snap (inverse modes, specialised kernel): every layer's output kept.
int run(df_chain* c, int mode, bool flow, const float* zin, const float* theta, float* xout, float* ldj, float* lp,
        double* sum_out, int64_t batch, void* stream, float* snap = nullptr, float* hsave = nullptr,
        int hsave_w = 0, int hsave_h = 0, float* fsave = nullptr);

}  // namespace api
}  // namespace df
