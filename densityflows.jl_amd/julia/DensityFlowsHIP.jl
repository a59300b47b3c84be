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

STATUS: written against include/densityflows_hip.h (ABI 1) but NOT executed —
there is no Julia toolchain in this build pipeline (SURVEY.md §8c).  The same
entry points are exercised from Python (densityflows.jl_amd/_lib.py) by the
parity tests.

Host `Array{Float32}` arguments are staged through device buffers
(df_device_alloc / df_memcpy_*); device arrays (AMDGPU.jl `ROCArray`) can be
passed by pointer to the same entry points without copies.
=#
module DensityFlowsHIP

using DensityFlows
import DensityFlows: forward, backward, forward!, FlowElement, CouplingLayer, CouplingBlock,
                     FlowChain, RNVPCouplingLayer, NICECouplingLayer, NormalizationLayer
import Flux

export HIPFlowChain, HIPTrainer, train_step!, train_step_graph!, trainables, copy_trainables!, hip_flow

const LIB = get(ENV, "DENSITYFLOWS_HIP_LIB", joinpath(@__DIR__, "..", "libdensityflows_hip.so"))
const ABI_VERSION = Int32(1)

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

mutable struct HIPFlowChain <: FlowElement
    handle::Ptr{Cvoid}
    d::Int
    n::Int
    keep::Vector{Any}               # host arrays the descriptor pointed to (until create returns)
end

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
    obj = HIPFlowChain(h[], d, max(n, 0), Any[])
    finalizer(c -> ccall((:df_chain_destroy, LIB), Cint, (Ptr{Cvoid},), c.handle), obj)
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

function _run(sym::Symbol, c::HIPFlowChain, y::Array{Float32,N}, θ::Array{Float32,N}) where {N}
    @assert size(y, 1) == c.d "input must be (d, dims...)"
    @assert size(θ, 1) == c.n "dimensions θ must match (n, dims...) with n number of trained parameters"
    B = prod(size(y)[2:N])
    out = similar(y); ldj = Array{Float32}(undef, size(y)[2:N]...)
    dy, dθ, dout, dl = _dev(sizeof(y)), _dev(sizeof(θ)), _dev(sizeof(y)), _dev(sizeof(ldj))
    try
        _h2d(dy, y); c.n > 0 && _h2d(dθ, θ)
        check(ccall((sym, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                    c.handle, dy, c.n > 0 ? dθ : C_NULL, dout, dl, B, C_NULL), String(sym))
        _d2h(out, dout); _d2h(ldj, dl)
    finally
        foreach(_free, (dy, dθ, dout, dl))
    end
    return out, ldj
end

forward(c::HIPFlowChain, z::Array{Float32,N}, θ::Array{Float32,N}) where {N} = _run(:df_chain_forward, c, z, θ)
backward(c::HIPFlowChain, x::Array{Float32,N}, θ::Array{Float32,N}) where {N} = _run(:df_chain_backward, c, x, θ)

function forward!(c::HIPFlowChain, z::Array{Float32,N}, θ::Array{Float32,N}) where {N}
    x, _ = _run(:df_chain_forward, c, z, θ)
    z .= x
    return nothing
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
end

"""Optimisers.setup(Adam(η, β, ϵ), model) on the device; the trainer owns the flat trainables."""
function HIPTrainer(c::HIPFlowChain; eta=1f-3, beta=(0.9f0, 0.999f0), epsilon=1f-8)
    t = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:df_train_create, LIB), Cint, (Ptr{Ptr{Cvoid}}, Ptr{Cvoid}, Ref{AdamDesc}),
                t, c.handle, AdamDesc(eta, beta[1], beta[2], epsilon)), "df_train_create")
    n = Ref{Int64}(0)
    check(ccall((:df_train_num_params, LIB), Cint, (Ptr{Cvoid}, Ref{Int64}), t[], n), "df_train_num_params")
    obj = HIPTrainer(t[], c, n[])
    finalizer(x -> ccall((:df_train_destroy, LIB), Cint, (Ptr{Cvoid},), x.handle), obj)
    return obj
end

"""One mini-batch step of train! (gradient of loss(backward(m, x, θ)) + Adam update)."""
function train_step!(t::HIPTrainer, x::Array{Float32,N}, θ::Array{Float32,N}) where {N}
    B = prod(size(x)[2:N])
    dx, dθ = _dev(sizeof(x)), _dev(max(sizeof(θ), 1))
    try
        _h2d(dx, x); t.chain.n > 0 && _h2d(dθ, θ)
        check(ccall((:df_train_step, LIB), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}),
                    t.handle, dx, t.chain.n > 0 ? dθ : C_NULL, B, C_NULL, C_NULL), "df_train_step")
    finally
        foreach(_free, (dx, dθ))
    end
    return nothing
end

"""
    train_step_graph!(t, x_dev, θ_dev, B)

train_step! on device buffers that stay the same across the mini-batch loop
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
