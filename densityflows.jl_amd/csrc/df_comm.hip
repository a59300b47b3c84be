// df_comm.hip — multi-GPU entry points of the C ABI (df_comm_*, df_flow_nll,
// df_train_allreduce_gradient, df_train_step_dist).
//
// One process per GPU.  The batch is split into contiguous sample shards
// (every sample is independent through the chain, src/Chains.jl:149-197), so
// the only exchanges are the ones the reference's reductions imply:
//   * loss = -mean(logpdf)               src/Flows.jl:352-359
//     → one RCCL all-reduce of {Σ logpdf (fp64), count} = 16 bytes;
//   * Flux.gradient over a batch         src/Flows.jl:398-411
//     → one RCCL all-reduce (sum) of the flat fp32 gradient, every rank having
//       taken the mean over the GLOBAL batch, before the identical Adam step.
//
// RCCL is resolved at run time (dlopen) instead of at link time: inside a
// PyTorch process the copy torch already loaded is reused (RTLD_NOLOAD by its
// NEEDED name), so one process never holds two RCCL instances; a Julia host
// gets /opt/rocm's librccl.so.1.  Without RCCL the library still loads and the
// df_comm_* calls return DF_ERR_UNSUPPORTED.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "densityflows_hip.h"
#include "df_handle.h"

using namespace df::api;

static_assert(sizeof(ncclUniqueId) == DF_COMM_ID_BYTES, "ncclUniqueId size");

namespace {

struct Rccl {
    void* handle = nullptr;
    std::string error;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*GetVersion)(int*) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl g_rccl;
std::once_flag g_rccl_once;

void load_rccl() {
    Rccl& r = g_rccl;
    const char* env = std::getenv("DF_RCCL_LIB");
    // Reuse a copy already in the process first (PyTorch's), then the system one.
    const char* noload[] = {"librccl.so", "librccl.so.1"};
    if (env && env[0]) r.handle = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    for (const char* n : noload)
        if (!r.handle) r.handle = dlopen(n, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
    const char* load[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : load)
        if (!r.handle) r.handle = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (!r.handle) {
        const char* e = dlerror();
        r.error = std::string("RCCL (librccl.so) could not be loaded: ") + (e ? e : "not found");
        return;
    }
#define DF_SYM(field, name)                                                     \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(r.handle, name));       \
    if (!r.field) {                                                             \
        r.error = std::string("RCCL symbol missing: ") + name;                 \
        return;                                                                 \
    }
    DF_SYM(GetUniqueId, "ncclGetUniqueId")
    DF_SYM(CommInitRank, "ncclCommInitRank")
    DF_SYM(CommDestroy, "ncclCommDestroy")
    DF_SYM(AllReduce, "ncclAllReduce")
    DF_SYM(GetVersion, "ncclGetVersion")
    DF_SYM(GetErrorString, "ncclGetErrorString")
#undef DF_SYM
}

const Rccl* rccl() {
    std::call_once(g_rccl_once, load_rccl);
    return g_rccl.error.empty() ? &g_rccl : nullptr;
}

int rccl_missing() { return set_err(DF_ERR_UNSUPPORTED, g_rccl.error); }

int nccl_err(const Rccl* r, ncclResult_t e, const char* where) {
    return set_err(DF_ERR_HIP, std::string(where) + ": " + r->GetErrorString(e));
}

__global__ void set_count_kernel(double* dst, double v) { *dst = v; }

}  // namespace

struct df_comm {
    ncclComm_t comm = nullptr;
    int rank = 0;
    int nranks = 1;
    int device = 0;
};

extern "C" {

int df_comm_get_unique_id(void* id_out) {
    if (!id_out) return set_err(DF_ERR_INVALID, "null id buffer");
    const Rccl* r = rccl();
    if (!r) return rccl_missing();
    ncclUniqueId id;
    ncclResult_t e = r->GetUniqueId(&id);
    if (e != ncclSuccess) return nccl_err(r, e, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return DF_OK;
}

int df_comm_init_rank(df_comm** out, int nranks, const void* id, int rank, int device) {
    if (!out || !id) return set_err(DF_ERR_INVALID, "null pointer");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return set_err(DF_ERR_INVALID, "invalid rank / number of ranks");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return set_err(DF_ERR_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return set_err(DF_ERR_INVALID, "device ordinal out of range");
    const Rccl* r = rccl();
    if (!r) return rccl_missing();
    DeviceGuard gd(device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    df_comm* c = new (std::nothrow) df_comm();
    if (!c) return set_err(DF_ERR_NOMEM, "host allocation failed");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclResult_t e = r->CommInitRank(&c->comm, nranks, uid, rank);  // collective over the nranks processes
    if (e != ncclSuccess) {
        delete c;
        return nccl_err(r, e, "ncclCommInitRank");
    }
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    *out = c;
    return DF_OK;
}

int df_comm_destroy(df_comm* c) {
    if (!c) return DF_OK;
    const Rccl* r = rccl();
    int rc = DF_OK;
    if (r && c->comm) {
        DeviceGuard gd(c->device);
        ncclResult_t e = r->CommDestroy(c->comm);
        if (e != ncclSuccess) rc = nccl_err(r, e, "ncclCommDestroy");
    }
    delete c;
    return rc;
}

int df_comm_get_info(const df_comm* c, int* rank, int* nranks, int* device) {
    if (!c) return set_err(DF_ERR_INVALID, "null communicator");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    if (device) *device = c->device;
    return DF_OK;
}

int df_comm_allreduce_sum(df_comm* c, void* buf, int64_t count, int dtype, void* stream) {
    if (!c) return set_err(DF_ERR_INVALID, "null communicator");
    if (count < 0) return set_err(DF_ERR_SHAPE, "negative element count");
    if (count == 0) return DF_OK;
    if (!buf) return set_err(DF_ERR_INVALID, "null buffer");
    ncclDataType_t t;
    if (dtype == DF_DTYPE_F32)
        t = ncclFloat32;
    else if (dtype == DF_DTYPE_F64)
        t = ncclFloat64;
    else
        return set_err(DF_ERR_INVALID, "dtype must be DF_DTYPE_F32 or DF_DTYPE_F64");
    const Rccl* r = rccl();
    if (!r) return rccl_missing();
    DeviceGuard gd(c->device);
    if (!gd.ok) return set_err(DF_ERR_HIP, "hipSetDevice failed");
    ncclResult_t e = r->AllReduce(buf, buf, (size_t)count, t, ncclSum, c->comm, static_cast<hipStream_t>(stream));
    return e == ncclSuccess ? DF_OK : nccl_err(r, e, "ncclAllReduce");
}

}  // extern "C"

namespace {
// {Σ logpdf, N} of this rank's shard, then the sum over the ranks; `flow`: θ raw
// (normalised with the chain's bounds) or as given
int nll(df_chain* chain, df_comm* comm, const float* x, const float* theta, int64_t batch, double* sum_count,
        void* stream, bool flow) {
    if (!chain) return set_err(DF_ERR_INVALID, "null chain");
    if (!sum_count) return set_err(DF_ERR_INVALID, "null {Σ, count} output");
    if (comm && comm->device != chain->device)
        return set_err(DF_ERR_INVALID, "communicator and chain are bound to different devices");
    int rc = flow ? df_flow_logpdf_sum(chain, x, theta, sum_count, batch, stream)
                  : df_chain_logpdf_sum(chain, x, theta, sum_count, batch, stream);
    if (rc != DF_OK) return rc;
    DeviceGuard gd(chain->device);
    hipLaunchKernelGGL(set_count_kernel, dim3(1), dim3(1), 0, static_cast<hipStream_t>(stream), sum_count + 1,
                       (double)batch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_err(e, "count kernel launch");
    return comm ? df_comm_allreduce_sum(comm, sum_count, 2, DF_DTYPE_F64, stream) : DF_OK;
}
}  // namespace

extern "C" {

int df_flow_nll(df_chain* chain, df_comm* comm, const float* x, const float* theta_raw, int64_t batch,
                double* sum_count, void* stream) {
    return nll(chain, comm, x, theta_raw, batch, sum_count, stream, true);
}

int df_chain_nll(df_chain* chain, df_comm* comm, const float* x, const float* theta, int64_t batch,
                 double* sum_count, void* stream) {
    return nll(chain, comm, x, theta, batch, sum_count, stream, false);
}

int df_train_allreduce_gradient(df_train* t, df_comm* comm, void* stream) {
    if (!t || !comm) return set_err(DF_ERR_INVALID, "null pointer");
    if (train_device(t) != comm->device)
        return set_err(DF_ERR_INVALID, "communicator and trainer are bound to different devices");
    float* g = nullptr;
    int64_t count = 0;
    int rc = df_train_grad_ptr(t, &g);
    if (rc == DF_OK) rc = df_train_num_params(t, &count);
    if (rc != DF_OK) return rc;
    return df_comm_allreduce_sum(comm, g, count, DF_DTYPE_F32, stream);
}

int df_train_step_dist(df_train* t, df_comm* comm, const float* x, const float* theta_raw, int64_t batch,
                       int64_t n_total, double* logpdf_sum, void* stream) {
    if (!t) return set_err(DF_ERR_INVALID, "null trainer");
    if (comm && train_device(t) != comm->device)
        return set_err(DF_ERR_INVALID, "communicator and trainer are bound to different devices");
    if (n_total < 1) return set_err(DF_ERR_INVALID, "n_total must be >= 1");
    int rc = df_train_gradient(t, x, theta_raw, batch, n_total, logpdf_sum, stream);
    if (rc != DF_OK) return rc;
    if (comm) {
        // ∇ and Σ logpdf (the caller's buffer or the handle's own, which the debug
        // check of df_train_apply reads): every rank then sees the global loss
        rc = df_train_allreduce_gradient(t, comm, stream);
        if (rc == DF_OK) rc = df_comm_allreduce_sum(comm, train_last_lpsum(t), 1, DF_DTYPE_F64, stream);
        if (rc != DF_OK) return rc;
    }
    return df_train_apply(t, stream);
}

}  // extern "C"
