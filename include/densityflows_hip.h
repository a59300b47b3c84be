/*
 * densityflows_hip.h — C ABI of the MI355X-native DensityFlows.jl hot path.
 *
 * The library (libdensityflows_hip.so, built for gfx950) evaluates a
 * DensityFlows.jl `FlowChain` of RealNVP / NICE coupling layers, coupling
 * blocks and NormalizationLayers over a batch of samples with fused HIP
 * kernels: the s/t conditioner MLPs run on f32 MFMA, the coupling transform,
 * the per-layer log-det-Jacobian (ldj) accumulation and the base-density
 * logpdf are fused behind them.
 *
 * Every entry point below replaces one Julia method of the reference
 * (DensityFlows.jl v1.0.0).  A Julia front-end binds them with `ccall`
 * (see INTEGRATION.md and densityflows.jl_amd/julia/DensityFlowsHIP.jl);
 * the Python host mirror binds them with ctypes.
 *
 * Conventions
 * -----------
 *  - Memory layout is exactly Julia's: a (d, B) Float32 matrix is
 *    column-major, so sample j occupies x[d*j .. d*j+d-1].  θ is (n, B), may
 *    be n = 0 (pointer may then be NULL).  ldj / logpdf are (B,).
 *  - Dense weights are Flux's `Dense.weight`: an (out, in) column-major
 *    Float32 matrix (W[i + out*k] = W_ik); `bias` has `out` entries or is
 *    NULL (`bias=false`).  Axes are Julia's 1-based index vectors.
 *  - Batch-compute calls take DEVICE pointers and a HIP stream (NULL = the
 *    default stream) and are stream-ordered (asynchronous w.r.t. the host).
 *  - All functions return DF_OK (0) or a negative df_status; the message of
 *    the last error on the calling thread is returned by df_last_error().
 *  - A df_chain handle is bound to one device and is not thread-safe;
 *    different handles may be used concurrently.
 */
#ifndef DENSITYFLOWS_HIP_H
#define DENSITYFLOWS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DF_ABI_VERSION 4

typedef enum df_status {
    DF_OK = 0,
    DF_ERR_INVALID = -1,     /* malformed descriptor / argument (Julia: ArgumentError) */
    DF_ERR_SHAPE = -2,       /* shape or rank mismatch (Julia: AssertionError / DimensionMismatch) */
    DF_ERR_HIP = -3,         /* HIP runtime error */
    DF_ERR_UNSUPPORTED = -4, /* structure outside the kernel's limits (see df_limits) */
    DF_ERR_NOMEM = -5,       /* device allocation failed */
    DF_ERR_NONFINITE = -6    /* a NaN/Inf was found where the caller asked for a check */
} df_status;

/* Activation functions σ of Flux.Dense (NNlib definitions). */
typedef enum df_act {
    DF_ACT_IDENTITY = 0,
    DF_ACT_RELU = 1,
    DF_ACT_TANH = 2,
    DF_ACT_SIGMOID = 3,
    DF_ACT_SOFTPLUS = 4,
    DF_ACT_LOGCOSH = 5,
    DF_ACT_LEAKYRELU = 6,  /* slope 0.01 */
    DF_ACT_ELU = 7,        /* α = 1 */
    DF_ACT_SWISH = 8
} df_act;

/* FlowElement kinds that the kernels evaluate. */
typedef enum df_layer_kind {
    DF_LAYER_RNVP = 0, /* RNVPCouplingLayer  (src/affine/RNVP.jl:41-48)          */
    DF_LAYER_NICE = 1, /* NICECouplingLayer  (src/affine/NICE.jl:31-36)          */
    DF_LAYER_NORM = 2  /* NormalizationLayer (src/norm/Normalization.jl:30-35)   */
} df_layer_kind;

/* One Flux.Dense(in, out, σ; bias).  src/Layers.jl:33-50. */
typedef struct df_dense_desc {
    int32_t in_dim;
    int32_t out_dim;
    int32_t act;        /* df_act */
    const float* W;     /* (out, in) column-major, host memory */
    const float* b;     /* out entries, or NULL for bias=false */
} df_dense_desc;

/* One flat layer of the chain.  CouplingBlocks (src/Blocks.jl:64-75) are
 * given as two consecutive layers with the same `element` index; the chain's
 * ldj is then accumulated exactly as the reference groups it:
 *   element ldj = ldj_1 .+ ldj_2            (src/Blocks.jl:136,149)
 *   chain ldj   = ldj_e1 .+ ldj_e2 .+ ...   (src/Chains.jl:160,179)          */
typedef struct df_layer_desc {
    int32_t kind;       /* df_layer_kind */
    int32_t element;    /* index of the FlowElement this layer belongs to */
    /* coupling layers: CouplingAxes (src/Axes.jl:28-35), 1-based */
    int32_t n_af;
    const int32_t* axis_af;  /* transformed dims, user (mask) order      */
    int32_t n_nn;
    const int32_t* axis_nn;  /* conditioner input rows of vcat(θ, z)     */
    int32_t n_dense_s;       /* 0 for NICE */
    const df_dense_desc* s_net;
    int32_t n_dense_t;
    const df_dense_desc* t_net;
    /* NormalizationLayer fields */
    const float* x_min;      /* d entries */
    const float* x_max;      /* d entries */
    float alpha;
    float beta;
} df_layer_desc;

typedef struct df_chain_desc {
    int32_t abi_version;     /* DF_ABI_VERSION */
    int32_t d;               /* data dimensions */
    int32_t n;               /* condition dimensions (0 = unconditional) */
    int32_t n_layers;
    const df_layer_desc* layers;
} df_chain_desc;

/* Structural limits of the fused kernels. */
typedef struct df_limits {
    int32_t max_state;       /* n + d                      */
    int32_t max_hidden;      /* widest hidden Dense        */
    int32_t max_af;          /* transformed dims per layer */
    int32_t max_layers;
} df_limits;

typedef struct df_chain_info {
    int32_t d, n, n_layers;
    int32_t hidden_tiles;         /* kernel variant: padded hidden width / 16 */
    int32_t samples_per_block;    /* samples one workgroup processes          */
    int32_t n_stages;             /* LDS weight stages per chain pass         */
    int64_t n_params;             /* trainable parameters (Flux.trainables)   */
    double flops_per_sample;      /* 2 × Σ Dense MACs (algorithmic)           */
    int64_t weight_bytes;         /* packed device weight blob                */
    int32_t kernel;               /* chain-pass kernel: 0 generic, 1 specialised,
                                     2 specialised relu-only, 3 FAST, 4 FAST on
                                     bf16x3 split stages (SPLIT), 5 wide,
                                     6 wide SPLIT                              */
    int32_t reserved;
    double split_flops_per_sample; /* part of flops_per_sample that kernels 4
                                      and 6 run as six bf16 products on MFMA */
} df_chain_info;

int df_get_abi_version(void);
const char* df_last_error(void);
int df_get_limits(df_limits* out);

/* ---- chain lifetime ------------------------------------------------------ */

typedef struct df_chain df_chain;

/* Validate and plan a descriptor without touching a device (the same checks
 * df_chain_create performs); fills `info` when non-NULL. */
int df_chain_validate(const df_chain_desc* desc, df_chain_info* info);

/* Build a device-resident chain (weights are copied and re-laid-out into MFMA
 * fragment order).  Replaces the Julia-side `FlowChain` object
 * (src/Chains.jl:78-80) for evaluation.  `device` = HIP device ordinal. */
int df_chain_create(df_chain** out, const df_chain_desc* desc, int device);
int df_chain_destroy(df_chain* chain);
int df_chain_get_info(const df_chain* chain, df_chain_info* out);

/* Replace the chain's parameters (Dense weights and biases, NormalizationLayer
 * bounds) with those of `desc`, which must describe the same structure (same
 * layers, axes, widths, activations and bias flags) — e.g. the model after
 * Optimisers.update! on the host, or one read by load_flow
 * (src/Loading.jl:324-376).  Synchronous.  Not allowed while df_train handles
 * are bound to the chain (they own the parameters: df_train_set_params). */
int df_chain_set_weights(df_chain* chain, const df_chain_desc* desc);

/* θ bounds of the Flow's MetaData (src/Data.jl:75-86; n floats each, host
 * memory).  Enables the df_flow_* entry points' in-kernel θ normalisation. */
int df_chain_set_theta_bounds(df_chain* chain, const float* theta_min, const float* theta_max);

/* ---- chain level (θ used as given) ---------------------------------------
 * forward(chain, z, θ)  -> (x, ldj)      src/Chains.jl:168-184
 * backward(chain, x, θ) -> (z, ldj)      src/Chains.jl:149-165
 * forward!(chain, z, θ)                  src/Chains.jl:187-197  (in place, no ldj)
 * `ldj` may be NULL (not written).  `x_out` may alias `z` for forward. */
int df_chain_forward(df_chain* chain, const float* z, const float* theta,
                     float* x_out, float* ldj_out, int64_t batch, void* stream);
int df_chain_backward(df_chain* chain, const float* x, const float* theta,
                      float* z_out, float* ldj_out, int64_t batch, void* stream);
int df_chain_forward_inplace(df_chain* chain, float* z, const float* theta,
                             int64_t batch, void* stream);

/* df_chain_logpdf / df_chain_logpdf_sum: the same quantities as df_flow_logpdf /
 * df_flow_logpdf_sum below with θ used as given — logpdf / loss of the MODEL,
 * as train! evaluates them on normalized_training_data (src/Flows.jl:391-392,
 * 419-430): backward(flow.model, x, t) then the MvNormal(0, I) log-density.
 * Independent of the chain's θ bounds. */
int df_chain_logpdf(df_chain* chain, const float* x, const float* theta,
                    float* logpdf_out, int64_t batch, void* stream);
int df_chain_logpdf_sum(df_chain* chain, const float* x, const float* theta,
                        double* sum_out, int64_t batch, void* stream);

/* ---- flow level (θ raw, normalised in-kernel with the stored bounds) -----
 * The @flow_wrapper methods (src/Macros.jl:104-112, applied at
 * src/DensityFlows.jl:72): f(flow, y, θ) = f(flow.model, y, normalize_input(θ)).
 * df_flow_logpdf: src/Flows.jl:272-281 — backward pass + MvNormal(0, I)
 * log-density + ldj, written per sample.
 * df_flow_logpdf_sum: Σ_j logpdf_j accumulated in fp64, deterministic
 * order, written to ONE double in device memory (the NLL partial that
 * src/Flows.jl:352-359 averages; all-reduced across GPUs by the caller). */
int df_flow_forward(df_chain* chain, const float* z, const float* theta_raw,
                    float* x_out, float* ldj_out, int64_t batch, void* stream);
int df_flow_backward(df_chain* chain, const float* x, const float* theta_raw,
                     float* z_out, float* ldj_out, int64_t batch, void* stream);
int df_flow_forward_inplace(df_chain* chain, float* z, const float* theta_raw,
                            int64_t batch, void* stream);
int df_flow_logpdf(df_chain* chain, const float* x, const float* theta_raw,
                   float* logpdf_out, int64_t batch, void* stream);
int df_flow_logpdf_sum(df_chain* chain, const float* x, const float* theta_raw,
                       double* sum_out, int64_t batch, void* stream);

/* ---- sampling ---------------------------------------------------------------
 * sample(flow, dims, θ) (src/Flows.jl:157-192): r ~ MvNormal(0, I) (Flows.jl:114)
 * drawn on the device, then forward!(flow, r, θ) — df_flow_forward_inplace, θ raw and
 * normalised in the kernel with the chain's bounds.  x_out: (d, batch) device memory;
 * for dims = (d1, d2, ...) pass batch = prod(dims) (the column-major (d, dims...) array
 * is the (d, batch) one).  theta_broadcast = 0: theta_raw is (n, batch); 1: theta_raw
 * is ONE n-vector used for every sample (the NTuple θ method, Flows.jl:178-188).
 * The draw: element k of the (d, batch) array comes from Philox4x32-10 with key =
 * seed and counter (offset + k/4, 0, 0, 0), word k%4; words (0,1), (2,3) are
 * Box-Muller pairs.  Julia's Xoshiro stream is not reproduced (by design);
 * df_random_normal returns the same draw on its own, so a caller can check
 * forward!(draw) against df_flow_sample with the same (seed, offset). */
int df_flow_sample(df_chain* chain, float* x_out, const float* theta_raw, int theta_broadcast, int64_t batch,
                   uint64_t seed, uint64_t offset, void* stream);
int df_random_normal(float* out, int64_t count, uint64_t seed, uint64_t offset, void* stream);

/* ---- training ---------------------------------------------------------------
 * train!(flow, data, opt_state; ...) src/Flows.jl:380-445: per batch
 *   grads = Flux.gradient(m -> loss(backward(m, x, θ)...), flow.model)   (:398-411)
 *   Optimisers.update!(opt_state, flow.model, grads[1])                  (:413)
 * with loss = -mean(logpdf(MvNormal(0, I), z) .+ ldj)  (src/Flows.jl:352-359)
 * and the custom pullbacks rrule(RNVP_backward) (src/affine/RNVP.jl:99-147),
 * rrule(NICE_backward) (src/affine/NICE.jl:84-113).
 *
 * A df_train handle owns the flat trainable parameters of its chain in
 * Flux.trainables order (per coupling layer: s_net then t_net; per Dense:
 * weight (out×in column-major) then bias; NormalizationLayer: none), the
 * Adam state and the gradient buffer, and rewrites the chain's packed
 * weights after every update, so df_chain_* / df_flow_* calls on the chain
 * see the trained parameters.  Supported: every chain df_chain_create accepts
 * (conditioner width <= 256, any depth — a single Dense included — e.g. the
 * hidden-256 config-5 model), with any of the nine DF_ACT_* activations; σ'
 * follows NNlib's derivative rules (from the output for relu / tanh_fast /
 * sigmoid_fast / leakyrelu / elu, from the pre-activation for softplus /
 * logcosh / swish).  Conditioners of the hidden <= 64, <= 4-output default
 * shape (_dflt_net, src/Layers.jl:33-50, n_sublayers <= 2) run one fused kernel
 * per net; the rest run the layer-wise MFMA path. */

typedef struct df_train df_train;

/* Optimisers.Adam(η, β, ϵ) (Optimisers.jl v0.4; defaults 1e-3, (0.9, 0.999), 1e-8) */
typedef struct df_adam {
    float eta;
    float beta1, beta2;
    float epsilon;
} df_adam;

/* Optimisers.setup(Adam(...), flow.model): state m = v = 0, βᵗ = β. */
int df_train_create(df_train** out, df_chain* chain, const df_adam* opt);
int df_train_destroy(df_train* t);
/* Form of the reverse sweep behind df_train_gradient.  Every form
 * computes the same gradient (rrule(RNVP_backward), src/affine/RNVP.jl:99-147, through
 * Flux.gradient, src/Flows.jl:398-411); df_train_create picks one from the chain:
 *   DF_SWEEP_FUSED      one fused per-net kernel: every conditioner the default
 *                       _dflt_net shape at hidden <= 64, <= 4 transformed dims;
 *   DF_SWEEP_H0FREE     layer-wise; the inverse pass keeps each net's features and H1,
 *                       the split dW1 recomputes H0: wide SPLIT chains whose nets are all
 *                       Dense(<= 32, 256, relu) → Dense(256, 256, relu) → Dense(256, <= 32);
 *   DF_SWEEP_KEPT       layer-wise; the inverse pass keeps every hidden activation
 *                       (chains on the generic or wide kernels, when they fit in half the
 *                       free device memory);
 *   DF_SWEEP_RECOMPUTE  layer-wise; the sweep recomputes the hidden activations.
 * H0FREE → KEPT → RECOMPUTE is also the fallback order when device memory runs short
 * (decided at the first gradient of each batch capacity). */
typedef enum df_sweep_form {
    DF_SWEEP_AUTO = 0,
    DF_SWEEP_FUSED = 1,
    DF_SWEEP_H0FREE = 2,
    DF_SWEEP_KEPT = 3,
    DF_SWEEP_RECOMPUTE = 4,
    /* request only: any layer-wise form (the library picks among the three above) */
    DF_SWEEP_LAYERWISE = 5,
    /* flag (with a layer-wise form): each net's dW products and the next net's
     * backward front as separate launches instead of merged ones (the same sums in
     * the same order: a bitwise A/B reference for the merged launches) */
    DF_SWEEP_SEPARATE = 16
} df_sweep_form;
/* df_train_create with a requested sweep form (DF_SWEEP_AUTO: as df_train_create).
 * A form the chain cannot take returns DF_ERR_UNSUPPORTED. */
int df_train_create_ex(df_train** out, df_chain* chain, const df_adam* opt, int sweep);
/* The form the trainer runs (before its first gradient: the one it will try first). */
int df_train_sweep(const df_train* t, int* form);
/* Number of trainable parameters (length of the flat vectors below). */
int df_train_num_params(const df_train* t, int64_t* count);
/* How the trainer's entry points (df_train_gradient and every step built on
 * it) read θ.  train! feeds the model normalised θ (normalized_training_data,
 * src/Data.jl:189-193, src/Flows.jl:391-392); a host may instead hand over the
 * raw θ and let the kernels normalise it with the Flow's MetaData bounds.
 *   DF_THETA_AUTO  (the default): normalise iff the chain has θ bounds
 *                  (df_chain_set_theta_bounds) at the time of the call;
 *   DF_THETA_RAW:  θ is raw and always normalised with the chain's bounds
 *                  (n > 0 without bounds: DF_ERR_INVALID);
 *   DF_THETA_GIVEN: θ is used as given (already normalised); the chain's
 *                  bounds are never consulted, so a later
 *                  df_chain_set_theta_bounds (e.g. by sample) cannot change
 *                  what this trainer computes.
 * A captured df_train_step_graph step is re-captured when the effective
 * convention changes. */
typedef enum df_theta_input {
    DF_THETA_AUTO = 0,
    DF_THETA_RAW = 1,
    DF_THETA_GIVEN = 2
} df_theta_input;
int df_train_set_theta_input(df_train* t, int mode);
/* Gradient of loss over this batch with the mean taken over `n_total`
 * samples (n_total = batch on one GPU; the global batch under data
 * parallelism, so the per-rank gradients SUM to the global one).  θ as the
 * trainer's df_theta_input says (default: normalised with the chain's
 * bounds when set).
 * The result is left in the device buffer returned by df_train_grad_ptr.
 * `logpdf_sum` (device double, may be NULL) receives Σ logpdf of the batch
 * at the current parameters (the loss before the update is -Σ/n_total). */
int df_train_gradient(df_train* t, const float* x, const float* theta_raw, int64_t batch, int64_t n_total,
                      double* logpdf_sum, void* stream);
/* Device pointer of the flat gradient (count floats); all-reduce it here
 * for multi-GPU data parallelism. */
int df_train_grad_ptr(df_train* t, float** grad_dev);
/* One Adam step with the current gradient; repacks the chain's weights. */
int df_train_apply(df_train* t, void* stream);
/* df_train_gradient (n_total = batch) followed by df_train_apply. */
int df_train_step(df_train* t, const float* x, const float* theta_raw, int64_t batch, double* logpdf_sum,
                  void* stream);
/* df_train_gradient (mean over n_total) + df_train_apply as ONE hipGraph
 * launch: the reverse sweep's per-net kernels, reduction, Adam and repack
 * are captured the second time the same (x, θ, batch, n_total, logpdf_sum)
 * buffers are seen and replayed from then on (the first call runs eagerly).
 * For train!'s mini-batch loop (src/Flows.jl:396-414) with reused device
 * staging buffers, where per-launch overhead dominates small batches.
 * Captures are dropped when a buffer they name is reallocated.  Not for
 * data parallelism (the gradient all-reduce sits between the two halves). */
int df_train_step_graph(df_train* t, const float* x, const float* theta_raw, int64_t batch, int64_t n_total,
                        double* logpdf_sum, void* stream);
/* train!(...; debug=true) (src/Flows.jl:404-409): when on, df_train_apply
 * (and the steps built on it) first reads the Σ logpdf of the last gradient
 * evaluation back to the host; if the loss is NaN or ±Inf the parameters are
 * NOT updated and DF_ERR_NONFINITE is returned (the reference throws an
 * ArgumentError before Optimisers.update!).  Costs one 8-byte device→host
 * copy and a stream synchronisation per step; df_train_step_graph runs its
 * steps eagerly while it is on. */
int df_train_set_debug(df_train* t, int on);
/* Copy the current trainables to / from host memory (count floats). */
int df_train_get_params(df_train* t, float* host_out, int64_t count);
int df_train_set_params(df_train* t, const float* host_in, int64_t count);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI ------------------------
 * The batch is sharded into contiguous sample blocks (samples are independent
 * through the chain, src/Chains.jl:149-197); the only exchanges are the sums
 * the reference's reductions imply:
 *   loss = -mean(logpdf)  (src/Flows.jl:352-359) → all-reduce {Σ logpdf, count}
 *   Flux.gradient          (src/Flows.jl:398-411) → all-reduce of the flat ∇
 * RCCL is resolved at run time (an already-loaded librccl is reused, else
 * librccl.so.1); without it these calls return DF_ERR_UNSUPPORTED.
 *
 * Bootstrap: rank 0 calls df_comm_get_unique_id and ships the
 * DF_COMM_ID_BYTES bytes to every rank out of band (MPI, a file, a TCP
 * store); then every rank calls df_comm_init_rank (collective). */

typedef struct df_comm df_comm;

#define DF_COMM_ID_BYTES 128

typedef enum df_dtype { DF_DTYPE_F32 = 0, DF_DTYPE_F64 = 1 } df_dtype;

int df_comm_get_unique_id(void* id_out /* DF_COMM_ID_BYTES */);
int df_comm_init_rank(df_comm** out, int nranks, const void* id, int rank, int device);
int df_comm_destroy(df_comm* comm);
int df_comm_get_info(const df_comm* comm, int* rank, int* nranks, int* device);
/* In-place sum over all ranks of `count` elements of device memory, ordered
 * on `stream`. */
int df_comm_allreduce_sum(df_comm* comm, void* buf_dev, int64_t count, int dtype, void* stream);
/* The NLL of a sharded batch (config 3): this rank's Σ logpdf of its shard
 * (df_flow_logpdf_sum) and its sample count are written to sum_count[0..1]
 * (device doubles) and all-reduced, so on return (stream-ordered) every rank
 * holds the global {Σ, N}; loss = -Σ / N.  comm = NULL: this process only. */
int df_flow_nll(df_chain* chain, df_comm* comm, const float* x, const float* theta_raw, int64_t batch,
                double* sum_count, void* stream);
/* df_flow_nll with θ used as given (normalised): the sharded loss of the model
 * on normalized data, as train!'s epoch losses (src/Flows.jl:419-430). */
int df_chain_nll(df_chain* chain, df_comm* comm, const float* x, const float* theta, int64_t batch,
                 double* sum_count, void* stream);
/* All-reduce (sum) of the flat gradient of df_train_gradient; every rank must
 * have called df_train_gradient with n_total = the global batch. */
int df_train_allreduce_gradient(df_train* t, df_comm* comm, void* stream);
/* One data-parallel train! step on this rank's shard: df_train_gradient (mean
 * over n_total, the global batch) → all-reduce of ∇ and of Σ logpdf →
 * df_train_apply (identical Adam step on every rank).  `logpdf_sum` (device
 * double or NULL) receives the GLOBAL Σ logpdf.  comm = NULL: one process. */
int df_train_step_dist(df_train* t, df_comm* comm, const float* x, const float* theta_raw, int64_t batch,
                       int64_t n_total, double* logpdf_sum, void* stream);

/* ---- diagnostics (no reference counterpart) ---------------------------------
 * Effective shader clock of the fused chain-pass kernels, the evidence behind a
 * clock-normalised benchmark time (the chip lowers its clock under load, and
 * devices differ).  on = 1 zeroes the stamp buffer and makes every later chain
 * pass of this handle that runs the specialised (kernels 1-4) or wide (5, 6)
 * kernel accumulate, per workgroup, Δs_memtime (shader cycles) and
 * Δs_memrealtime (100 MHz ticks) over its wave 0's lifetime; on = 0 stops.
 * df_chain_clock_read synchronises the device and returns the median over
 * workgroup slots and the ratio of sums (GHz), and the number of slots
 * stamped (0: nothing stamped yet). */
int df_chain_clock_probe(df_chain* chain, int on);
int df_chain_clock_read(df_chain* chain, double* ghz_median, double* ghz_mean, int64_t* n_slots);

/* ---- device memory helpers (for hosts without a GPU array package) ------ */
int df_device_alloc(void** ptr, size_t bytes);
int df_device_free(void* ptr);
int df_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int df_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int df_stream_synchronize(void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DENSITYFLOWS_HIP_H */
