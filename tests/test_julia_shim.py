"""Static checks of the Julia front-end binding (densityflows.jl_amd/julia/DensityFlowsHIP.jl).

There is no Julia toolchain here or on the GPU box, so the shim is
checked as text against the two things it must agree with:
  * the C ABI (include/densityflows_hip.h): every ccall'd symbol is declared there with
    the same argument count, and the ABI version the shim checks at load is the header's;
  * the reference's method table (src/Flows.jl, src/Chains.jl): each shim method that
    replaces a reference method is strictly more specific in the flow/model argument and
    equal in the others, so the reference's own calls dispatch to it without ambiguity.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "densityflows.jl_amd", "julia", "DensityFlowsHIP.jl")
HEADER = os.path.join(ROOT, "include", "densityflows_hip.h")


@pytest.fixture(scope="module")
def shim():
    with open(SHIM) as f:
        return f.read()


@pytest.fixture(scope="module")
def header_decls():
    """name -> parameter count of every function the header declares."""
    with open(HEADER) as f:
        text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(?:int|const char\*)\s+(df_\w+)\s*\(([^)]*)\)\s*;", text):
        params = m.group(2).strip()
        decls[m.group(1)] = 0 if params in ("", "void") else len(params.split(","))
    return decls


def _ccalls(text):
    """(symbol, number of argument types) of every ccall((:sym, LIB), ret, (types...), ...)."""
    out = []
    for m in re.finditer(r"ccall\(\(:(\w+), LIB\),\s*[\w{}]+,\s*\(", text):
        i, depth = m.end(), 1
        start = i
        while depth:
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        types = text[start:i - 1].strip()
        n = 0 if types == "" else len([t for t in re.split(r",(?![^{]*})", types) if t.strip()])
        out.append((m.group(1), n))
    return out


def test_every_ccall_matches_the_header(shim, header_decls):
    calls = _ccalls(shim)
    assert len(calls) >= 20
    for sym, n in calls:
        assert sym in header_decls, f"{sym} is not declared in include/densityflows_hip.h"
        assert n == header_decls[sym], f"{sym}: ccall passes {n} argument types, the header declares {header_decls[sym]}"


def test_abi_version_checked_at_load(shim):
    with open(HEADER) as f:
        v = int(re.search(r"#define DF_ABI_VERSION (\d+)", f.read()).group(1))
    assert re.search(rf"const ABI_VERSION = Int32\({v}\)", shim)
    init = re.search(r"function __init__\(\)(.*?)\nend", shim, re.S)
    assert init and "df_get_abi_version" in init.group(1) and "ABI_VERSION" in init.group(1)


def test_train_bang_is_strictly_more_specific_than_the_reference(shim):
    # reference: train!(flow::Flow{T}, data::DataArrays{T}, optimiser_state::NamedTuple; ...) (src/Flows.jl:380-389)
    assert re.search(r"function train!\(flow::Flow\{T,D,N,<:HIPModel\}, data::DataArrays\{T\}, "
                     r"optimiser_state::NamedTuple;", shim)
    # every train! method types its third argument (an untyped one would be ambiguous)
    for m in re.finditer(r"^(?:function )?train!\((\w+::[^;)]*)[;)]", shim, re.M):
        args = [a.strip() for a in re.split(r",(?![^{]*})", m.group(1))]
        assert len(args) == 3 and all("::" in a for a in args), m.group(0)
        assert args[0].startswith("flow::Flow{T,D,N,<:HIPModel}"), m.group(0)
        assert args[2].split("::")[1] in ("NamedTuple", "Optimisers.AbstractRule", "HIPTrainer"), m.group(0)


def test_optimiser_rule_reaches_the_device(shim):
    # Optimisers.setup(rule, model) must yield a Leaf holding the user's rule ...
    assert "Optimisers.trainable(c::HIPFlowChain) = (; params = c.params)" in shim
    # ... and a state without one is refused, never replaced by a default Adam()
    body = re.search(r"function _state_rule\(state\)(.*?)\nend", shim, re.S).group(1)
    assert "throw(ArgumentError" in body and "Optimisers.Adam()" not in body


def test_trainer_lifetime_follows_the_chain(shim):
    assert "_TRAINERS" not in shim and "IdDict" not in shim
    fin = re.search(r"finalizer\(obj\) do c(.*?)end", shim, re.S).group(1)
    assert "_destroy!(c.trainer)" in fin and fin.index("_destroy!") < fin.index("df_chain_destroy")


@pytest.mark.parametrize("fn", ["forward", "backward", "forward!", "logpdf_sum", "train_step!", "flow_nll",
                                "train_step_dist!"])
def test_array_arguments_accept_views(shim, fn):
    """normalized_training_data returns selectdim views (src/Data.jl:185-193): every
    host-array entry point takes AbstractArray{Float32,N} and copies views."""
    sigs = re.findall(rf"^(?:function )?{re.escape(fn)}\(([^=]*?)\) where \{{N\}}", shim, re.M | re.S)
    assert sigs, fn
    for sig in sigs:
        assert "Array{Float32,N}" in sig
        assert re.search(r"(?<!Abstract)Array\{Float32,N\}", sig) is None, sig


def test_sample_methods_narrow_the_flow_only(shim):
    # reference: sample(rng, flow::Flow{T,D}, dims::NTuple{M,Integer}, θ::AbstractArray{T,K})
    #            sample(rng, flow::Flow{T,D,N}, dims::Tuple{Vararg{Integer}}, θ::NTuple{N,T})  (src/Flows.jl:159-188)
    assert re.search(r"function sample\(rng::Random\.AbstractRNG, flow::Flow\{T,D,N,<:HIPModel\}, "
                     r"dims::NTuple\{M,Integer\},\s*θ::AbstractArray\{T,K\}", shim)
    assert re.search(r"sample\(rng::Random\.AbstractRNG, flow::Flow\{T,D,N,<:HIPModel\}, "
                     r"dims::Tuple\{Vararg\{Integer\}\},\s*θ::NTuple\{N,T\}\)", shim)
    assert ":df_flow_sample" in shim


def _julia_ccalls_by_function(text):
    """Julia function name -> literal ccall symbols of its methods, in source order."""
    text = re.sub(r'"""(.*?)"""', lambda m: "\n" * m.group(0).count("\n"), text, flags=re.S)
    lines = text.split("\n")
    out, i = {}, 0
    while i < len(lines):
        ln = lines[i]
        m = re.match(r"function ([\w!]+)\(", ln)
        if m:
            j = i + 1
            while lines[j] != "end":
                j += 1
        else:
            m = re.match(r"([A-Za-z_][\w!]*)\(", ln)
            if not m:
                i += 1
                continue
            j = i + 1
            while j < len(lines) and lines[j][:1] in (" ", "\t"):
                j += 1
            j -= 1
        body = "\n".join(lines[i:j + 1])
        out.setdefault(m.group(1), []).extend(re.findall(r"ccall\(\(:(\w+), LIB\)", body))
        i = j + 1
    return {k: v for k, v in out.items() if v}


def _replay_ccalls_by_function():
    import ast

    path = os.path.join(ROOT, "tests", "julia_replay.py")
    with open(path) as f:
        tree = ast.parse(f.read())
    out = {}
    for node in tree.body:
        if not isinstance(node, ast.FunctionDef):
            continue
        calls = [c for c in ast.walk(node) if isinstance(c, ast.Call) and isinstance(c.func, ast.Name)
                 and c.func.id == "cc" and c.args and isinstance(c.args[0], ast.Constant)]
        calls.sort(key=lambda c: (c.lineno, c.col_offset))
        if calls:
            out[node.name] = [c.args[0].value for c in calls]
    return out


def test_replay_issues_the_shims_ccalls(shim):
    """tests/julia_replay.py (run on the GPU by test_gpu_julia_replay.py) re-enacts
    each shim function: the same literal ccall symbols in the same order."""
    jl = _julia_ccalls_by_function(shim)
    py = _replay_ccalls_by_function()
    assert len(jl) >= 20, sorted(jl)
    for name, syms in jl.items():
        pyname = name.replace("!", "_bang")
        assert pyname in py, f"{name} has no replay in tests/julia_replay.py"
        assert py[pyname] == syms, f"{name}: shim {syms}, replay {py[pyname]}"
    assert set(py) <= {n.replace("!", "_bang") for n in jl}, sorted(set(py) - {n.replace("!", "_bang") for n in jl})


def test_model_level_calls_take_theta_as_given(shim):
    """The θ contract: model-level entry points never read the
    chain's θ bounds — only sample goes through a df_flow_* entry point."""
    jl = _julia_ccalls_by_function(shim)
    for name in ("logpdf_sum", "flow_nll", "train_step!", "train_step_dist!", "train_step_graph!"):
        assert not any(s.startswith("df_flow_") for s in jl[name]), (name, jl[name])
    assert jl["HIPTrainer"][-1] == "df_train_set_theta_input"
    assert re.search(r"df_train_set_theta_input, LIB\), Cint, \(Ptr\{Cvoid\}, Cint\), t\[\], DF_THETA_GIVEN\)", shim)
    assert re.search(r"const DF_THETA_GIVEN = Cint\(2\)", shim)
    flow_syms = {s for v in jl.values() for s in v if s.startswith("df_flow_")}
    assert flow_syms == {"df_flow_sample"}, flow_syms


def test_weight_export_walks_flux_trainables(shim):
    """copy_trainables! and hip_flow call no C entry point, so the ccall replay check
    above does not see them.  The order contract, statically:
      * HIPFlowChain hands the device the model's parameters as
        vcat(vec.(Flux.trainables(chain))) and copy_trainables! writes them back with the
        same walk over Flux.trainables(model), column-major copyto! per array, checking
        the total length;
      * tests/julia_replay.py has a replay of copy_trainables! (run on the GPU by
        test_gpu_julia_replay.py: trained vector → fresh model → re-created chain,
        bitwise the trained chain's forward / backward);
      * hip_flow goes through the reference's own reader (DensityFlows.load_flow,
        src/Loading.jl:348-377) and wraps f.model as FlowChain((HIPFlowChain(f.model),)).
    """
    import ast

    body = re.search(r"function copy_trainables!\(model::FlowChain, p::Vector\{Float32\}\)(.*?)\nend", shim, re.S)
    assert body, "copy_trainables! not found"
    b = body.group(1)
    assert re.search(r"for a in Flux\.trainables\(model\)", b)
    assert "copyto!(a, 1, p, off + 1, n)" in b and "off += n" in b
    assert re.search(r"off == length\(p\) \|\| throw\(DimensionMismatch", b)
    hc = re.search(r"function HIPFlowChain\(chain::FlowChain;.*?\nend", shim, re.S)
    assert hc and re.search(r"reduce\(vcat, \[vec\(Float32\.\(a\)\) for a in Flux\.trainables\(chain\)\]\)", hc.group(0))
    hf = re.search(r"function hip_flow\(directory::AbstractString;.*?\nend", shim, re.S)
    assert hf and "DensityFlows.load_flow(directory)" in hf.group(0)
    assert "FlowChain((HIPFlowChain(f.model; device = device),))" in hf.group(0)
    with open(os.path.join(ROOT, "tests", "julia_replay.py")) as f:
        tree = ast.parse(f.read())
    names = {n.name for n in tree.body if isinstance(n, ast.FunctionDef)}
    assert "copy_trainables_bang" in names
