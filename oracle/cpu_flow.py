"""TEST INFRASTRUCTURE: ctypes front of oracle/cpu_flow.cpp, the C++/OpenMP CPU
restatement of FlowChain.forward (src/Chains.jl:168-184).  Used by tests/
(pinned against the numpy oracle, flow_oracle.py) and by bench.py's
cpu_baseline leg; never by the product path."""
import ctypes
import os

import numpy as np

from . import flow_oracle as O

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_ACTS = {"identity": 0, "relu": 1, "tanh": 2, "sigmoid": 3, "softplus": 4, "logcosh": 5, "leakyrelu": 6,
         "elu": 7, "swish": 8}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libcpu_flow.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/libcpu_flow.so is not built (make -C oracle)")
        L = ctypes.CDLL(path)
        for name, T in (("cpu_flow_forward_f32", ctypes.c_float), ("cpu_flow_forward_f64", ctypes.c_double)):
            f = getattr(L, name)
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        L.cpu_flow_max_threads.restype = ctypes.c_int
        _LIB = L
    return _LIB


def compile_spec(spec, d, n, dtype=np.float32):
    """Pre-order program + parameter stream of a spec dict (flow_oracle format)."""
    prog, par = [], []

    def net(ns):
        prog.append(len(ns))
        for D in ns:
            W = np.asarray(D["W"], np.float64)
            b = D.get("b")
            prog.extend([W.shape[1], W.shape[0], _ACTS[D["act"]], 0 if b is None else 1])
            par.extend(W.ravel(order="F"))
            if b is not None:
                par.extend(np.asarray(b, np.float64))

    def walk(e):
        k = e["kind"]
        if k == "chain":
            prog.extend([0, len(e["layers"])])
            for c in e["layers"]:
                walk(c)
        elif k == "block":
            prog.append(1)
            walk(e["layer_1"])
            walk(e["layer_2"])
        elif k in ("rnvp", "nice"):
            prog.append(2 if k == "rnvp" else 3)
            af = [a - 1 for a in e["axis_af"]]
            nn = [a - 1 for a in e["axis_nn"]]
            prog.extend([len(af)] + af + [len(nn)] + nn)
            net(e["s_net"] if k == "rnvp" else [])
            net(e["t_net"])
        elif k == "norm":
            prog.append(4)
            par.extend(np.asarray(e["x_min"], np.float64))
            par.extend(np.asarray(e["x_max"], np.float64))
            par.extend([float(e["alpha"]), float(e["beta"])])
            par.append(float(O._norm_ldj_const(e, np.dtype(dtype).type)))  # ldj constant in the pass's dtype
        else:
            raise ValueError(k)

    walk(spec)
    return np.asarray(prog, np.int32), np.asarray(par, np.float64)


class CPUFlow:
    """forward(z, θ) → (x, ldj) on the host cores, fp32 (the timed proxy) or fp64."""

    def __init__(self, spec, d, n, dtype=np.float32):
        self.prog, self.par = compile_spec(spec, d, n, dtype)
        self.d, self.n, self.dtype = d, n, np.dtype(dtype)
        self.fn = lib().cpu_flow_forward_f32 if self.dtype == np.float32 else lib().cpu_flow_forward_f64

    def forward(self, z, theta=None, threads=0, out=None):
        z = np.ascontiguousarray(np.asarray(z, self.dtype).T)  # (B, d) rows = Julia (d, B) columns
        B = z.shape[0]
        th = np.ascontiguousarray(np.asarray(theta, self.dtype).T) if self.n else np.zeros((B, 1), self.dtype)
        x = np.empty_like(z) if out is None else out[0]
        ldj = np.empty(B, self.dtype) if out is None else out[1]
        rc = self.fn(self.prog.ctypes.data, self.par.ctypes.data, self.d, self.n, z.ctypes.data, th.ctypes.data,
                     x.ctypes.data, ldj.ctypes.data, B, int(threads))
        assert rc == 0
        return x.T, ldj


def max_threads():
    return int(lib().cpu_flow_max_threads())
