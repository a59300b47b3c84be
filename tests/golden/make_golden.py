"""Generate golden vectors for the GPU parity tests from the CPU oracle.

The reference (Julia/Flux) cannot run in this pipeline, so the
expected outputs are the oracle's fp64 evaluation (oracle/flow_oracle.py, pinned
against the reference's own invariant tests in tests/test_oracle.py) on
seeded weights and inputs.  Re-running this script must reproduce the committed
files bit for bit (tests/test_oracle.py::test_golden_regenerates checks it).

Configs (BASELINE.json / SURVEY.md §8d):
  cfg1  d=5, n=1: 3 RNVP layers, masks [1,2,3],[3,4,5],[5,1,2], hidden 16, relu,
        + NormalizationLayer(datatest x, -1, 1) (README / test/runtests.jl:105-110);
        θ from test/datatest.jld2 values {-1, 2}.  B = 4096.
  cfg2  d=5, n=0: FlowChain(CouplingBlock, 4, 5; hidden 64) = 8 RNVP layers.  B = 4096.
  cfg4  d=32, n=8: FlowChain(CouplingBlock, 8, 32; n=8, hidden 256) = 16 layers.  B = 1024.
        Weights are regenerated from the seed (9.8 MB would not fit a fixture);
        a checksum of them is stored.
Biases are drawn U(-0.1, 0.1) so the bias path is exercised (Flux inits zeros).
cfg2/cfg4 scale the final Dense of every conditioner by 0.1 so that the
8/16-layer random-init flows stay finite (exp(s) overflows otherwise).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import flow_oracle as O  # noqa: E402


def cfg1_spec(seed=11):
    rng = np.random.default_rng(seed)
    x = np.load(os.path.join(HERE, "datatest_x.npy"))
    layers = [O.rnvp_layer(rng, O.coupling_axes(5, m, n=1), n_sub=2, hidden=16, bias_scale=0.1)
              for m in ([1, 2, 3], [3, 4, 5], [5, 1, 2])]
    layers.append(O.normalization_layer(x, -1.0, 1.0))
    return {"kind": "chain", "layers": layers}


def blocks_spec(d, n, nblocks, hidden, seed, out_scale=0.1):
    rng = np.random.default_rng(seed)
    ax = O.coupling_axes_cut(d, d // 2, n=n)
    return {"kind": "chain", "layers": [O.coupling_block(rng, ax, n_sub=2, hidden=hidden, bias_scale=0.1,
                                                         out_scale=out_scale)
                                        for _ in range(nblocks)]}


def cfg2_spec(seed=22):
    return blocks_spec(5, 0, 4, 64, seed)


def cfg4_spec(seed=44):
    return blocks_spec(32, 8, 8, 256, seed)


def spec_to_arrays(spec, prefix="", out=None):
    """Serialise a spec to (structure JSON, {key: array})."""
    out = {} if out is None else out
    k = spec["kind"]
    if k == "chain":
        return {"kind": "chain", "layers": [spec_to_arrays(l, f"{prefix}{i}_", out)[0]
                                            for i, l in enumerate(spec["layers"])]}, out
    if k == "block":
        return {"kind": "block", "layer_1": spec_to_arrays(spec["layer_1"], prefix + "a_", out)[0],
                "layer_2": spec_to_arrays(spec["layer_2"], prefix + "b_", out)[0]}, out
    if k == "norm":
        out[prefix + "xmin"] = np.asarray(spec["x_min"], np.float32)
        out[prefix + "xmax"] = np.asarray(spec["x_max"], np.float32)
        return {"kind": "norm", "alpha": spec["alpha"], "beta": spec["beta"],
                "x_min": prefix + "xmin", "x_max": prefix + "xmax"}, out
    s = {key: spec[key] for key in ("kind", "d", "n", "axis_id", "axis_af", "axis_nn")}
    for net in ("s_net", "t_net"):
        if net not in spec:
            continue
        s[net] = []
        for j, D in enumerate(spec[net]):
            kw, kb = f"{prefix}{net}{j}_W", f"{prefix}{net}{j}_b"
            out[kw] = np.asarray(D["W"], np.float32)
            if D.get("b") is not None:
                out[kb] = np.asarray(D["b"], np.float32)
            s[net].append({"W": kw, "b": kb if D.get("b") is not None else None, "act": D["act"]})
    return s, out


def arrays_to_spec(struct, arrs):
    k = struct["kind"]
    if k == "chain":
        return {"kind": "chain", "layers": [arrays_to_spec(l, arrs) for l in struct["layers"]]}
    if k == "block":
        return {"kind": "block", "layer_1": arrays_to_spec(struct["layer_1"], arrs),
                "layer_2": arrays_to_spec(struct["layer_2"], arrs)}
    if k == "norm":
        return {"kind": "norm", "alpha": struct["alpha"], "beta": struct["beta"],
                "x_min": arrs[struct["x_min"]], "x_max": arrs[struct["x_max"]]}
    s = dict(struct)
    for net in ("s_net", "t_net"):
        if net in struct:
            s[net] = [{"W": arrs[D["W"]], "b": arrs[D["b"]] if D["b"] else None, "act": D["act"]}
                      for D in struct[net]]
    return s


def weights_checksum(spec):
    _, arrs = spec_to_arrays(spec)
    acc = np.float64(0)
    for i, key in enumerate(sorted(arrs)):
        a = arrs[key].astype(np.float64).ravel()
        acc += np.sum(a * np.cos(np.arange(a.size) * 0.001 + i))
    return float(acc)


def make(name, spec, d, n, B, seed, store_weights, theta_kind):
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((d, B)).astype(np.float32)
    if theta_kind == "datatest":
        th_raw = np.where(rng.random((n, B)) < 0.5, -1.0, 2.0).astype(np.float32)
        tmin, tmax = np.full(n, -1, np.float32), np.full(n, 2, np.float32)
    else:
        th_raw = rng.uniform(-1.0, 2.0, (n, B)).astype(np.float32)
        tmin, tmax = np.full(n, -1, np.float32), np.full(n, 2, np.float32)
    th = O.normalize_input(th_raw, tmin, tmax) if n > 0 else np.zeros((0, B), np.float32)
    x, ldj_f = O.forward(spec, z, th, np.float64)
    # an independent point set for the inverse: x_in = fp32 forward output
    x_in = x.astype(np.float32)
    z_b, ldj_b = O.backward(spec, x_in, th, np.float64)
    lp = O.flow_logpdf(spec, x_in, th, np.float64)
    out = {"z": z, "theta_raw": th_raw, "theta": th, "theta_min": tmin, "theta_max": tmax,
           "x_fwd": x, "ldj_fwd": ldj_f, "x_in": x_in, "z_bwd": z_b, "ldj_bwd": ldj_b, "logpdf": lp}
    struct, arrs = spec_to_arrays(spec)
    meta = {"name": name, "d": d, "n": n, "B": B, "seed": seed, "struct": struct,
            "weights_checksum": weights_checksum(spec), "weights_stored": store_weights}
    if store_weights:
        for k, v in arrs.items():
            out["w_" + k] = v
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = os.path.join(HERE, f"golden_{name}.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path))


def load(name):
    f = np.load(os.path.join(HERE, f"golden_{name}.npz"), allow_pickle=False)
    meta = json.loads(bytes(f["meta"]).decode())
    if meta["weights_stored"]:
        arrs = {k[2:]: f[k] for k in f.files if k.startswith("w_")}
        spec = arrays_to_spec(meta["struct"], arrs)
    else:
        spec = {"cfg4": cfg4_spec}[name]()
    return spec, {k: f[k] for k in f.files if not k.startswith("w_")}, meta


def main():
    make("cfg1", cfg1_spec(), 5, 1, 4096, 101, True, "datatest")
    make("cfg2", cfg2_spec(), 5, 0, 4096, 202, True, None)
    make("cfg4", cfg4_spec(), 32, 8, 1024, 404, False, "uniform")


if __name__ == "__main__":
    main()
