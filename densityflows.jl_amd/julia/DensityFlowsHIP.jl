#=
DensityFlowsHIP.jl — Julia front-end binding of libdensityflows_hip.so.

Drop-in for the DensityFlows.jl hot path: `HIPFlowChain <: FlowElement` is
built from an existing `FlowChain` (src/Chains.jl:78-80) and implements the
reference's plugin contract (docs/src/documentation.md:172-192):

    forward(::HIPFlowChain, z, θ)  -> (x, ldj)     src/Chains.jl:168-184
    backward(::HIPFlowChain, x, θ) -> (z, ldj)     src/Chains.jl:149-165
    forward!(::HIPFlowChain, z, θ)                 src/Chains.jl:187-197

so `Flow`'s @flow_wrapper methods (src/Macros.jl:104-112), `logpdf`
(src/Flows.jl:272-281) and `sample` (src/Flows.jl:157-192) run on the MI355X
unchanged once the chain is wrapped: `FlowChain((HIPFlowChain(chain),))`.

STATUS: written against include/densityflows_hip.h (ABI 4; `__init__` refuses a
library of another ABI) but NOT executed — there is no Julia toolchain in this
build pipeline (SURVEY.md §8c).  Not executed in particular: the Functors walk
that `Optimisers.setup(Adam(η), flow.model)` makes over HIPFlowChain (declared
below with `@functor HIPFlowChain (params,)`), `hip_flow` / `load_flow` and
`copy_trainables!`.  What IS executed on the GPU: tests/julia_replay.py replays,
ccall for ccall, the C-call sequence of this file's HIPFlowChain, forward /
backward, logpdf_sum, HIPTrainer, train_step!, _hip_train!, _set_bounds! and
_hip_sample (tests/test_gpu_julia_replay.py, against the oracle's epoch loop),
and tests/test_julia_shim.py checks statically that the replay issues the
same ccall symbols in the same order as each of those functions here, that
every ccall matches the header, and the method signatures against the
reference's (dispatch specificity, AbstractArray inputs).

θ CONTRACT.  Model-level calls take θ as given, as the reference's model
methods do (train! normalises once, src/Flows.jl:391-392): forward / backward /
forward! (df_chain_*), logpdf_sum (df_chain_logpdf_sum), flow_nll
(df_chain_nll) and every HIPTrainer step (created with DF_THETA_GIVEN, so
the chain's θ bounds never reach them).  Flow-level calls take raw θ and
normalise it in the kernel with the Flow's MetaData bounds: only `sample`
(df_flow_sample after _set_bounds!), matching @flow_wrapper
(src/Macros.jl:104-112).

Host `Array{Float32}` arguments are staged through device buffers
(df_device_alloc / df_memcpy_*); device arrays (AMDGPU.jl `ROCArray`) can be
passed by pointer to the same entry points without copies.
=#
module DensityFlowsHIP

using DensityFlows
import DensityFlows: forward, backward, forward!, train!, sample, FlowElement, CouplingLayer, CouplingBlock,
                     FlowChain, RNVPCouplingLayer, NICECouplingLayer, NormalizationLayer, Flow, DataArrays
import Distributions, LinearAlgebra, Random
import Flux, Optimisers

export HIPFlowChain, HIPTrainer, HIPComm, train_step!, train_step_graph!, train_step_dist!, trainables,
       copy_trainables!, hip_flow, flow_nll, sample

const LIB = get(ENV, "DENSITYFLOWS_HIP_LIB", joinpath(@__DIR__, "..", "libdensityflows_hip.so"))
const ABI_VERSION = Int32(4)

function __init__()
    v = ccall((:df_get_abi_version, LIB), Cint, ())
    v == ABI_VERSION || error("$LIB has ABI version $v, this binding needs $ABI_VERSION")
end

# ---- C structs (include/densityflows_hip.h) --------------------------------
struct DenseDesc                 # df_dense_desc
    in_dim::Int32
    out_dim::Int32
    act::Int32
    W::Ptr{Float32}
    b::Ptr{Float32}
end

struct LayerDesc                 # df_layer_desc
    kind::Int32
    element::Int32
    n_af::Int32
    axis_af::Ptr{Int32}
    n_nn::Int32
    axis_nn::Ptr{Int32}
    n_dense_s::Int32
    s_net::Ptr{DenseDesc}
    n_dense_t::Int32
    t_net::Ptr{DenseDesc}
    x_min::Ptr{Float32}
    x_max::Ptr{Float32}
    alpha::Float32
    beta::Float32
end

struct ChainDesc                 # df_chain_desc
    abi_version::Int32
    d::Int32
    n::Int32
    n_layers::Int32
    layers::Ptr{LayerDesc}
end

const ACT = Dict{Any,Int32}(identity => 0, Flux.relu => 1, tanh => 2, Flux.tanh_fast => 2,
                            Flux.sigmoid => 3, Flux.sigmoid_fast => 3, Flux.softplus => 4,
                            Flux.logcosh => 5, Flux.leakyrelu => 6, Flux.elu => 7, Flux.swish => 8)

lasterror() = unsafe_string(ccall((:df_last_error, LIB), Cstring, ()))

function check(rc::Integer, what::AbstractString)
    rc == 0 && return nothing
    msg = "$what: " * lasterror()
    rc == -1 && throw(ArgumentError(msg))           # DF_ERR_INVALID
    rc == -2 && throw(DimensionMismatch(msg))       # DF_ERR_SHAPE
    throw(ErrorException("densityflows_hip [$rc] $msg"))
end

# Device staging buffers of one handle, grown on demand and reused across calls
# (a host-array call costs the copies, not four allocations).
mutable struct Staging
    ptr::Vector{Ptr{Cvoid}}
    bytes::Vector{Int}
end
Staging(n::Integer) = Staging(fill(C_NULL, n), zeros(Int, n))

function _buf!(st::Staging, i::Integer, bytes::Integer)
    if st.bytes[i] < bytes
        st.ptr[i] == C_NULL || _free(st.ptr[i])
        st.ptr[i] = C_NULL; st.bytes[i] = 0
        st.ptr[i] = _dev(bytes); st.bytes[i] = max(bytes, 1)
    end
    return st.ptr[i]
end
_release!(st::Staging) = (foreach(p -> p == C_NULL || _free(p), st.ptr); fill!(st.ptr, C_NULL); fill!(st.bytes, 0))

mutable struct HIPFlowChain <: FlowElement
    handle::Ptr{Cvoid}
    d::Int
    n::Int
    keep::Vector{Any}               # host arrays the descriptor pointed to (until create returns)
    stage::Staging                  # [y, θ, out, ldj, Σ]
    params::Vector{Float32}         # host copy of the trainables (Flux.trainables order): what
                                    # Optimisers.setup sees, so the rule it wraps reaches train!
    trainer::Any                    # the device trainer of this chain (Nothing or HIPTrainer)
    trainer_key::Any                # its Adam hyper-parameters
    bounds::Any                     # θ bounds last given to df_chain_set_theta_bounds
end

# Optimisers.setup(rule, FlowChain((HIPFlowChain(chain),))) yields a Leaf holding `rule`:
# the chain is a functor whose only child is the flat parameter vector (the handle,
# staging buffers and trainer are not walked), and that child is its trainable
Optimisers.Functors.@functor HIPFlowChain (params,)
Optimisers.trainable(c::HIPFlowChain) = (; params = c.params)

# flatten the chain into (element index, layer) pairs; blocks share an element
function _flatten(chain::FlowChain)
    out = Tuple{Int,Any}[]
    for (e, el) in enumerate(chain.layers)
        if el isa CouplingBlock
            push!(out, (e - 1, el.layer_1)); push!(out, (e - 1, el.layer_2))
        elseif el isa FlowChain
            for (_, l) in _flatten(el); push!(out, (e - 1, l)); end
        else
            push!(out, (e - 1, el))
        end
    end
    return out
end

function _net(keep, net::Flux.Chain)
    descs = DenseDesc[]
    for D in net.layers
        W = Matrix{Float32}(D.weight)                 # (out, in) column-major, as Flux stores it
        push!(keep, W)
        b = D.bias isa AbstractVector ? Vector{Float32}(D.bias) : nothing
        b === nothing || push!(keep, b)
        act = get(ACT, D.σ) do
            throw(ArgumentError("activation $(D.σ) has no fused kernel"))
        end
        push!(descs, DenseDesc(size(W, 2), size(W, 1), act, pointer(W),
                               b === nothing ? Ptr{Float32}(0) : pointer(b)))
    end
    push!(keep, descs)
    return Int32(length(descs)), pointer(descs)
end

function HIPFlowChain(chain::FlowChain; device::Integer = 0)
    keep = Any[]
    flat = _flatten(chain)
    d = n = -1
    layers = LayerDesc[]
    for (e, l) in flat
        if l isa NormalizationLayer
            xmn = Vector{Float32}(l.x_min); xmx = Vector{Float32}(l.x_max); push!(keep, xmn, xmx)
            d = length(xmn)
            push!(layers, LayerDesc(2, e, 0, C_NULL, 0, C_NULL, 0, C_NULL, 0, C_NULL,
                                    pointer(xmn), pointer(xmx), l.α, l.β))
        else
            ax = l.axes
            d, n = ax.d, ax.n
            af = Vector{Int32}(ax.axis_af); nn = Vector{Int32}(ax.axis_nn); push!(keep, af, nn)
            ns, ps = l isa RNVPCouplingLayer ? _net(keep, l.s_net) : (Int32(0), Ptr{DenseDesc}(0))
            nt, pt = _net(keep, l.t_net)
            push!(layers, LayerDesc(l isa RNVPCouplingLayer ? 0 : 1, e, length(af), pointer(af),
                                    length(nn), pointer(nn), ns, ps, nt, pt, C_NULL, C_NULL, 0f0, 0f0))
        end
    end
    push!(keep, layers)
    desc = Ref(ChainDesc(ABI_VERSION, d, max(n, 0), length(layers), pointer(layers)))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve keep begin
        check(ccall((:df_chain_create, LIB), Cint, (Ptr{Ptr{Cvoid}}, Ref{ChainDesc}, Cint),
                    h, desc, device), "df_chain_create")
    end
    params = isempty(Flux.trainables(chain)) ? Float32[] :
             reduce(vcat, [vec(Float32.(a)) for a in Flux.trainables(chain)])
    obj = HIPFlowChain(h[], d, max(n, 0), Any[], Staging(5), params, nothing, nothing, nothing)
    finalizer(obj) do c
        _release!(c.stage)
        c.trainer === nothing || _destroy!(c.trainer)   # df_chain_destroy needs its trainers gone
        ccall((:df_chain_destroy, LIB), Cint, (Ptr{Cvoid},), c.handle)
    end
    return obj
end

# ---- host-array staging -----------------------------------------------------
function _dev(bytes)
    p = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:df_device_alloc, LIB), Cint, (Ptr{Ptr{Cvoid}}, Csize_t), p, max(bytes, 1)), "df_device_alloc")
    return p[]
end
_free(p) = ccall((:df_device_free, LIB), Cint, (Ptr{Cvoid},), p)
_h2d(dst, src::Array) = check(ccall((:df_memcpy_h2d, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                                    dst, src, sizeof(src), C_NULL), "h2d")
_d2h(dst::Array, src) = check(ccall((:df_memcpy_d2h, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                                    dst, src, sizeof(dst), C_NULL), "d2h")

# device calls take contiguous column-major arrays; views (selectdim in
# normalized_training_data, src/Data.jl:185-193) are copied first
_dense(a::Array{Float32}) = a
_dense(a::AbstractArray{Float32}) = Array{Float32}(a)

function _run(sym::Symbol, c::HIPFlowChain, y::AbstractArray{Float32,N}, θ::AbstractArray{Float32,N}) where {N}
    y, θ = _dense(y), _dense(θ)
    @assert size(y, 1) == c.d "input must be (d, dims...)"
    @assert size(θ, 1) == c.n "dimensions θ must match (n, dims...) with n number of trained parameters"
    B = prod(size(y)[2:N])
    out = similar(y); ldj = Array{Float32}(undef, size(y)[2:N]...)
    dy, dθ = _buf!(c.stage, 1, sizeof(y)), _buf!(c.stage, 2, sizeof(θ))
    dout, dl = _buf!(c.stage, 3, sizeof(y)), _buf!(c.stage, 4, sizeof(ldj))
    _h2d(dy, y); c.n > 0 && _h2d(dθ, θ)
    check(ccall((sym, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                c.handle, dy, c.n > 0 ? dθ : C_NULL, dout, dl, B, C_NULL), String(sym))
    _d2h(out, dout); _d2h(ldj, dl)
    return out, ldj
end

forward(c::HIPFlowChain, z::AbstractArray{Float32,N}, θ::AbstractArray{Float32,N}) where {N} =
    _run(:df_chain_forward, c, z, θ)
backward(c::HIPFlowChain, x::AbstractArray{Float32,N}, θ::AbstractArray{Float32,N}) where {N} =
    _run(:df_chain_backward, c, x, θ)

"""forward!(c, z, θ): src/Chains.jl:187-197 — z overwritten by the chain's output
(df_chain_forward_inplace: one staging buffer, no ldj)."""
function forward!(c::HIPFlowChain, z::AbstractArray{Float32,N}, θ::AbstractArray{Float32,N}) where {N}
    zz, θ = _dense(z), _dense(θ)
    @assert size(z, 1) == c.d "input must be (d, dims...)"
    @assert size(θ, 1) == c.n "dimensions θ must match (n, dims...) with n number of trained parameters"
    B = prod(size(z)[2:N])
    dz, dθ = _buf!(c.stage, 1, sizeof(zz)), _buf!(c.stage, 2, sizeof(θ))
    _h2d(dz, zz); c.n > 0 && _h2d(dθ, θ)
    check(ccall((:df_chain_forward_inplace, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                c.handle, dz, c.n > 0 ? dθ : C_NULL, B, C_NULL), "df_chain_forward_inplace")
    _d2h(zz, dz)
    zz === z || copyto!(z, zz)
    return nothing
end

"""Σ_j logpdf_j (fp64, on the device) of the chain's inverse pass under MvNormal(0, I):
the sum src/Flows.jl:352-359 averages.  θ as given (already normalised, as
normalized_training_data returns it): df_chain_logpdf_sum, whatever bounds the
chain holds."""
function logpdf_sum(c::HIPFlowChain, x::AbstractArray{Float32,N}, θ::AbstractArray{Float32,N}) where {N}
    x, θ = _dense(x), _dense(θ)
    B = prod(size(x)[2:N])
    dx, dθ, ds = _buf!(c.stage, 1, sizeof(x)), _buf!(c.stage, 2, sizeof(θ)), _buf!(c.stage, 5, 16)
    _h2d(dx, x); c.n > 0 && _h2d(dθ, θ)
    check(ccall((:df_chain_logpdf_sum, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                c.handle, dx, c.n > 0 ? dθ : C_NULL, ds, B, C_NULL), "df_chain_logpdf_sum")
    r = Vector{Float64}(undef, 1)
    _d2h(r, ds)
    return r[1]
end

# ---- training: train! (src/Flows.jl:380-445) on the device ----------------------
struct AdamDesc                  # df_adam
    eta::Float32
    beta1::Float32
    beta2::Float32
    epsilon::Float32
end

mutable struct HIPTrainer
    handle::Ptr{Cvoid}
    chain::HIPFlowChain
    n_params::Int
    stage::Staging                  # [x, θ, Σ logpdf]
end

function _destroy!(t::HIPTrainer)
    t.handle == C_NULL && return nothing
    _release!(t.stage)
    ccall((:df_train_destroy, LIB), Cint, (Ptr{Cvoid},), t.handle)
    t.handle = C_NULL
    return nothing
end

"""Optimisers.setup(Adam(η, β, ϵ), model) on the device; the trainer owns the flat trainables.
Its steps take θ as given (DF_THETA_GIVEN: normalised, as train! passes it to the model)."""
function HIPTrainer(c::HIPFlowChain; eta=1f-3, beta=(0.9f0, 0.999f0), epsilon=1f-8)
    t = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:df_train_create, LIB), Cint, (Ptr{Ptr{Cvoid}}, Ptr{Cvoid}, Ref{AdamDesc}),
                t, c.handle, AdamDesc(eta, beta[1], beta[2], epsilon)), "df_train_create")
    n = Ref{Int64}(0)
    check(ccall((:df_train_num_params, LIB), Cint, (Ptr{Cvoid}, Ref{Int64}), t[], n), "df_train_num_params")
    check(ccall((:df_train_set_theta_input, LIB), Cint, (Ptr{Cvoid}, Cint), t[], DF_THETA_GIVEN),
          "df_train_set_theta_input")
    obj = HIPTrainer(t[], c, n[], Staging(3))
    finalizer(_destroy!, obj)
    return obj
end

"""One mini-batch step of train! (gradient of loss(backward(m, x, θ)) + Adam update),
θ as given (normalised).  Returns the batch loss before the update (−Σ logpdf / B)."""
function train_step!(t::HIPTrainer, x::AbstractArray{Float32,N}, θ::AbstractArray{Float32,N}) where {N}
    x, θ = _dense(x), _dense(θ)
    B = prod(size(x)[2:N])
    dx, dθ, ds = _buf!(t.stage, 1, sizeof(x)), _buf!(t.stage, 2, sizeof(θ)), _buf!(t.stage, 3, 8)
    _h2d(dx, x); t.chain.n > 0 && _h2d(dθ, θ)
    rc = ccall((:df_train_step, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}),
               t.handle, dx, t.chain.n > 0 ? dθ : C_NULL, B, ds, C_NULL)
    r = Vector{Float64}(undef, 1)
    rc == DF_ERR_NONFINITE || check(rc, "df_train_step")
    _d2h(r, ds)
    l = Float32(-r[1] / B)
    rc == DF_ERR_NONFINITE && throw(NonFiniteLoss(l))
    return l
end

const DF_ERR_NONFINITE = Cint(-6)
const DF_THETA_GIVEN = Cint(2)      # df_theta_input

"""The debug check of df_train_step refused an update (NaN / Inf loss)."""
struct NonFiniteLoss <: Exception
    loss::Float32
end

"""
    train_step_graph!(t, x_dev, θ_dev, B)

train_step! (θ as given) on device buffers that stay the same across the mini-batch loop
(copy each batch into them): the step is captured as one hipGraph the second
time the buffers repeat and replayed afterwards (df_train_step_graph).
"""
function train_step_graph!(t::HIPTrainer, x::Ptr{Float32}, θ::Ptr{Float32}, B::Integer; stream = C_NULL)
    check(ccall((:df_train_step_graph, LIB), Cint,
                (Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32}, Int64, Int64, Ptr{Cvoid}, Ptr{Cvoid}),
                t.handle, x, θ, B, B, C_NULL, stream), "df_train_step_graph")
    return nothing
end

"""Flux.trainables order: per coupling layer s_net then t_net, per Dense vec(weight) then bias."""
function trainables(t::HIPTrainer)
    p = Vector{Float32}(undef, t.n_params)
    check(ccall((:df_train_get_params, LIB), Cint, (Ptr{Cvoid}, Ptr{Float32}, Int64), t.handle, p, t.n_params),
          "df_train_get_params")
    return p
end

"""
    set_debug!(t::HIPTrainer, on::Bool)

train!(...; debug = true) (src/Flows.jl:404-409): a NaN / Inf batch loss makes the
step refuse the Adam update (df_train_set_debug → DF_ERR_NONFINITE).
"""
set_debug!(t::HIPTrainer, on::Bool) =
    check(ccall((:df_train_set_debug, LIB), Cint, (Ptr{Cvoid}, Cint), t.handle, on), "df_train_set_debug")

# ---- multi-GPU: RCCL communicator (df_comm_*), one Julia process per GPU ----------
mutable struct HIPComm
    handle::Ptr{Cvoid}
    rank::Int
    nranks::Int
    stage::Staging                  # [{Σ, N}]
end

"""128 opaque bytes (ncclUniqueId) made on rank 0 and shipped to every rank out of band."""
function comm_unique_id()
    id = zeros(UInt8, 128)
    check(ccall((:df_comm_get_unique_id, LIB), Cint, (Ptr{UInt8},), id), "df_comm_get_unique_id")
    return id
end

"""HIPComm(nranks, id, rank; device): ncclCommInitRank over the nranks processes (collective)."""
function HIPComm(nranks::Integer, id::Vector{UInt8}, rank::Integer; device::Integer = 0)
    length(id) == 128 || throw(ArgumentError("unique id must be 128 bytes"))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:df_comm_init_rank, LIB), Cint, (Ptr{Ptr{Cvoid}}, Cint, Ptr{UInt8}, Cint, Cint),
                h, nranks, id, rank, device), "df_comm_init_rank")
    obj = HIPComm(h[], rank, nranks, Staging(1))
    finalizer(obj) do c
        _release!(c.stage)
        ccall((:df_comm_destroy, LIB), Cint, (Ptr{Cvoid},), c.handle)
    end
    return obj
end

"""
    flow_nll(c::HIPFlowChain, comm, x_shard, θ_shard) -> loss

Config 3's sharded NLL, `loss = -mean(logpdf)` (src/Flows.jl:352-359) over the
union of every rank's shard: df_chain_nll all-reduces {Σ logpdf, N} over RCCL.
θ as given (already normalised, as train!'s epoch losses take it); the chain's
bounds are not consulted.  `comm = nothing`: this process only.
"""
function flow_nll(c::HIPFlowChain, comm::Union{HIPComm,Nothing}, x::AbstractArray{Float32,N},
                  θ::AbstractArray{Float32,N}) where {N}
    x, θ = _dense(x), _dense(θ)
    B = prod(size(x)[2:N])
    dx, dθ, ds = _buf!(c.stage, 1, sizeof(x)), _buf!(c.stage, 2, sizeof(θ)), _buf!(c.stage, 5, 16)
    _h2d(dx, x); c.n > 0 && _h2d(dθ, θ)
    check(ccall((:df_chain_nll, LIB), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}),
                c.handle, comm === nothing ? C_NULL : comm.handle, dx, c.n > 0 ? dθ : C_NULL, B, ds, C_NULL),
          "df_chain_nll")
    r = Vector{Float64}(undef, 2)
    _d2h(r, ds)
    return Float32(-r[1] / r[2])
end

"""
    train_step_dist!(t, comm, x_shard, θ_shard, n_total)

One data-parallel train! step (θ as given, normalised): this rank's gradient with
the mean over the global batch `n_total`, RCCL all-reduce of ∇ and Σ logpdf, the identical Adam step on
every rank (df_train_step_dist).  Returns the global batch loss before the update.
"""
function train_step_dist!(t::HIPTrainer, comm::HIPComm, x::AbstractArray{Float32,N}, θ::AbstractArray{Float32,N},
                          n_total::Integer) where {N}
    x, θ = _dense(x), _dense(θ)
    B = prod(size(x)[2:N])
    dx, dθ, ds = _buf!(t.stage, 1, sizeof(x)), _buf!(t.stage, 2, sizeof(θ)), _buf!(t.stage, 3, 8)
    _h2d(dx, x); t.chain.n > 0 && _h2d(dθ, θ)
    rc = ccall((:df_train_step_dist, LIB), Cint,
               (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Int64, Ptr{Cvoid}, Ptr{Cvoid}),
               t.handle, comm.handle, dx, t.chain.n > 0 ? dθ : C_NULL, B, n_total, ds, C_NULL)
    rc == DF_ERR_NONFINITE || check(rc, "df_train_step_dist")
    r = Vector{Float64}(undef, 1)
    _d2h(r, ds)
    l = Float32(-r[1] / n_total)
    rc == DF_ERR_NONFINITE && throw(NonFiniteLoss(l))
    return l
end

# ---- train! drop-in (src/Flows.jl:380-445) ------------------------------------------
const HIPModel = FlowChain{<:Tuple{HIPFlowChain}}

_adam(rule::Optimisers.Adam) = (Float32(rule.eta), (Float32(rule.beta[1]), Float32(rule.beta[2])),
                                Float32(rule.epsilon))
_adam(::Any) = throw(ArgumentError("the device optimiser is Optimisers.Adam"))

# The device trainer of a chain lives on the chain (created on first use, replaced when
# the Adam hyper-parameters change), so its lifetime — and its device moments — follow
# the chain's; the chain's finalizer destroys it first.
function _trainer!(c::HIPFlowChain, rule)
    η, β, ϵ = _adam(rule)
    key = (η, β, ϵ)
    if c.trainer === nothing || c.trainer_key != key
        c.trainer === nothing || _destroy!(c.trainer)
        c.trainer = HIPTrainer(c; eta = η, beta = β, epsilon = ϵ)
        c.trainer_key = key
    end
    return c.trainer
end

# The rule inside Optimisers.setup(rule, flow.model): HIPFlowChain exposes its flat
# trainables (Optimisers.trainable), so the state tree holds one Leaf with the user's
# rule.  A state without a Leaf was not built from this model: refuse it.
function _state_rule(state)
    rules = Any[]
    Optimisers.fmap(x -> (x isa Optimisers.Leaf && push!(rules, x.rule); x), state;
                    exclude = x -> x isa Optimisers.Leaf)
    isempty(rules) && throw(ArgumentError("optimiser state holds no Optimisers.Leaf: build it with " *
                                          "Optimisers.setup(Adam(η), flow.model) on the HIP-wrapped model"))
    all(r -> r == rules[1], rules) || throw(ArgumentError("one Adam rule per HIP chain"))
    return rules[1]
end

"""
    train!(flow, data, opt; epochs=100, batchsize=64, shuffle=true, verbose=true, debug=false)

src/Flows.jl:380-445 for a Flow whose model is `FlowChain((HIPFlowChain(chain),))`:
the same DataLoader over `normalized_training_data` (batchsize, partial last batch,
shuffle), one device step per batch (df_train_step: inverse pass, reverse sweep,
Adam, weight repack), then the full-set train / valid losses pushed to
`flow.train_loss` / `flow.valid_loss` per epoch (fp64 device Σ logpdf).  `opt` is
`Optimisers.setup(Adam(η), flow.model)`, an `Optimisers.Adam` rule or a
`HIPTrainer`.  `debug`: a NaN/Inf batch loss prints and throws ArgumentError
before the update (as the reference); a NaN/Inf epoch loss prints and returns
`(z, ldj)` of that set; returns `(nothing, nothing)` at the end.
Copy the trained parameters into a Julia model with `copy_trainables!`.
"""
# The reference method is train!(flow::Flow{T}, data::DataArrays{T}, optimiser_state::NamedTuple; ...)
# (src/Flows.jl:380-389).  This one is strictly more specific (argument 1 narrower, the
# others equal), so the reference's own call `train!(flow, data, Optimisers.setup(Adam(η),
# flow.model))` dispatches here without ambiguity.
function train!(flow::Flow{T,D,N,<:HIPModel}, data::DataArrays{T}, optimiser_state::NamedTuple;
                kws...) where {T,D,N}
    c = flow.model.layers[1]
    return _hip_train!(flow, data, _trainer!(c, _state_rule(optimiser_state)); kws...)
end

# An Optimisers rule or a HIPTrainer directly (argument 3 disjoint from NamedTuple: no
# ambiguity with the reference method).
train!(flow::Flow{T,D,N,<:HIPModel}, data::DataArrays{T}, rule::Optimisers.AbstractRule; kws...) where {T,D,N} =
    _hip_train!(flow, data, _trainer!(flow.model.layers[1], rule); kws...)

function train!(flow::Flow{T,D,N,<:HIPModel}, data::DataArrays{T}, t::HIPTrainer; kws...) where {T,D,N}
    t.chain === flow.model.layers[1] || throw(ArgumentError("trainer of another chain"))
    return _hip_train!(flow, data, t; kws...)
end

function _hip_train!(flow::Flow{T,D,N}, data::DataArrays{T}, t::HIPTrainer; epochs::Int = 100,
                     batchsize::Int = 64, shuffle::Bool = true, verbose::Bool = true,
                     debug::Bool = false) where {T,D,N}
    flow.base isa Distributions.MvNormal && all(iszero, Distributions.mean(flow.base)) &&
        Distributions.cov(flow.base) == LinearAlgebra.diagm(ones(T, D)) ||
        throw(ArgumentError("the device loss is the MvNormal(0, I) base of Flow(model, data)"))
    c = flow.model.layers[1]
    set_debug!(t, debug)
    train_data = DensityFlows.normalized_training_data(data, flow.metadata)
    valid_data = DensityFlows.normalized_validation_data(data, flow.metadata)
    loader = Flux.DataLoader(train_data; batchsize = batchsize, shuffle = shuffle)
    setloss(set) = Float32(-logpdf_sum(c, set...) / prod(size(set[1])[2:end]))
    for _ ∈ 1:epochs
        for (x_batch, t_batch) ∈ loader
            try
                train_step!(t, x_batch, t_batch)
            catch e
                e isa NonFiniteLoss || rethrow()
                copyto!(c.params, trainables(t))   # the last good parameters, as update! left them
                z, ldj = backward(c, x_batch, t_batch)
                println("$(e.loss), $ldj, $z")
                throw(ArgumentError(""))
            end
        end
        train_loss = setloss(train_data)
        push!(flow.train_loss, train_loss)
        if debug && ((train_loss != train_loss) || isinf(train_loss))
            println("Problem with train loss $train_loss")
            copyto!(c.params, trainables(t))
            return backward(c, train_data...)
        end
        valid_loss = setloss(valid_data)
        push!(flow.valid_loss, valid_loss)
        if debug && ((valid_loss != valid_loss) || isinf(valid_loss))
            println("Problem with valid loss $valid_loss")
            copyto!(c.params, trainables(t))
            return backward(c, valid_data...)
        end
        verbose && println("epoch: $(length(flow.train_loss)) | train_loss = $train_loss, valid_loss = $valid_loss")
    end
    copyto!(c.params, trainables(t))               # host mirror of the trained parameters
    debug && return nothing, nothing
    return nothing
end

# ---- sample (src/Flows.jl:157-192) on the device ----------------------------------
function _set_bounds!(c::HIPFlowChain, md)
    c.n == 0 && return nothing
    b = (Vector{Float32}(md.θ_min), Vector{Float32}(md.θ_max))
    c.bounds == b && return nothing
    check(ccall((:df_chain_set_theta_bounds, LIB), Cint, (Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32}),
                c.handle, b[1], b[2]), "df_chain_set_theta_bounds")
    c.bounds = b
    return nothing
end

# r ~ MvNormal(0, I) drawn on the device (Philox4x32-10 keyed by 64 bits of `rng`, so a
# seeded rng reproduces the sample; Julia's own Xoshiro stream is not reproduced), then
# forward!(flow, r, θ) with θ normalised in the kernel: one df_flow_sample call.
function _hip_sample(rng::Random.AbstractRNG, flow::Flow, dims::Tuple, θ::Array{Float32}, bcast::Bool)
    c = flow.model.layers[1]
    _set_bounds!(c, flow.metadata)
    B = prod(dims)
    r = Array{Float32}(undef, c.d, dims...)
    dr, dθ = _buf!(c.stage, 3, sizeof(r)), _buf!(c.stage, 2, sizeof(θ))
    c.n > 0 && _h2d(dθ, θ)
    check(ccall((:df_flow_sample, LIB), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, UInt64, UInt64, Ptr{Cvoid}),
                c.handle, dr, c.n > 0 ? dθ : C_NULL, bcast ? 1 : 0, B, rand(rng, UInt64), 0, C_NULL),
          "df_flow_sample")
    _d2h(r, dr)
    return r
end

# The reference methods are sample(rng, flow::Flow{T,D}, dims::NTuple{M,Integer},
# θ::AbstractArray{T,K}) and sample(rng, flow::Flow{T,D,N}, dims::Tuple{Vararg{Integer}},
# θ::NTuple{N,T}) (src/Flows.jl:159-188); these narrow argument 2 only, and the
# convenience methods (Integer dims, default rng, :190-195) dispatch to them.
function sample(rng::Random.AbstractRNG, flow::Flow{T,D,N,<:HIPModel}, dims::NTuple{M,Integer},
                θ::AbstractArray{T,K} = DensityFlows.dflt_θ(T, dims)) where {T,D,N,M,K}
    @assert K == M + 1 "dimensions θ must match (n, dims...) with n number of trained parameters"
    @assert size(θ, 1) == N && size(θ)[2:end] == Tuple(dims) "dimensions θ must match (n, dims...) with n number of trained parameters"
    return _hip_sample(rng, flow, Tuple(dims), _dense(Float32.(θ)), false)
end

sample(rng::Random.AbstractRNG, flow::Flow{T,D,N,<:HIPModel}, dims::Tuple{Vararg{Integer}},
       θ::NTuple{N,T}) where {T,D,N} = _hip_sample(rng, flow, Tuple(dims), Float32[θ...], true)

"""
    copy_trainables!(model::FlowChain, p::Vector{Float32})

Write the device-trained flat parameters `p` (`trainables(t)`, Flux.trainables
order) back into the Julia model, so the reference's own `save_flow` /
`save_element` (src/Loading.jl:78-96, 124-173, 324-346) persist them.
"""
function copy_trainables!(model::FlowChain, p::Vector{Float32})
    off = 0
    for a in Flux.trainables(model)
        n = length(a)
        copyto!(a, 1, p, off + 1, n)
        off += n
    end
    off == length(p) || throw(DimensionMismatch("model has $off trainables, device vector $(length(p))"))
    return model
end

"""
    hip_flow(directory; device = 0) -> Flow

Weight import through the reference's own JLD2 reader: `load_flow(directory)`
(src/Loading.jl:348-377) rebuilds the Flow that `save_flow` wrote, then its
model is wrapped as `FlowChain((HIPFlowChain(model),))` (src/Chains.jl:78-80),
so `logpdf`, `sample` and the @flow_wrapper methods of the returned Flow run on
the MI355X.  Metadata, base distribution and loss histories are kept.
"""
function hip_flow(directory::AbstractString; device::Integer = 0)
    f = DensityFlows.load_flow(directory)
    hip = FlowChain((HIPFlowChain(f.model; device = device),))
    T = eltype(f.metadata.θ_min)
    return DensityFlows.Flow{T, f.metadata.d, f.metadata.n, typeof(hip), typeof(f.base), typeof(f.metadata.θ_min)}(
        hip, f.base, f.metadata, f.train_loss, f.valid_loss)
end

end # module
