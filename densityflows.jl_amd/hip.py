"""HIP executor: compiles a flow element into a ``df_chain`` handle and runs
the fused kernels on device arrays.

Array convention (mirrors the reference): a batch is an array of logical
shape ``(d, dims...)`` in Julia memory order (column-major: each sample's d
values are contiguous).  torch tensors whose *reversed-axes view* is
contiguous are used zero-copy; anything else (numpy arrays, other strides) is
copied once into that layout.  Outputs are returned with the same logical
shape, as column-major views of a fresh contiguous buffer.

PyTorch is used only as plumbing (device allocation, streams).  There is no
CPU fallback: without the native library or a GPU every call raises.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Tuple

import numpy as np

from . import _lib
from .layers import (CouplingBlock, NICECouplingLayer, NormalizationLayer, RNVPCouplingLayer)

__all__ = ["HIPChain", "flatten_elements", "as_julia_device", "julia_empty", "chain_dims"]


def _torch():
    import torch  # plumbing only

    return torch


# ---------------------------------------------------------------------------
# layout helpers
# ---------------------------------------------------------------------------

def julia_empty(rows: int, dims: Tuple[int, ...], device):
    """A column-major (rows, dims...) float32 tensor: returns (flat buffer, logical view)."""
    torch = _torch()
    shape_rev = tuple(reversed(dims)) + (rows,)
    buf = torch.empty(shape_rev, dtype=torch.float32, device=device)
    nd = len(shape_rev)
    view = buf.permute(*reversed(range(nd)))
    return buf.reshape(-1), view


def as_julia_device(a, rows: int, device, name: str = "array"):
    """Return (flat contiguous device buffer in Julia order, dims, was_numpy)."""
    torch = _torch()
    was_numpy = not isinstance(a, torch.Tensor)
    if was_numpy:
        a = np.asarray(a, dtype=np.float32)
        if a.ndim < 1 or a.shape[0] != rows:
            raise _lib.DimensionMismatch(f"{name} must have size ({rows}, dims...), got {a.shape}")
        # Julia memory order = Fortran order of the logical array
        host = np.asfortranarray(a).ravel(order="K")
        t = torch.from_numpy(np.ascontiguousarray(host)).to(device)
        return t, tuple(a.shape[1:]), True
    if a.dtype != torch.float32:
        raise _lib.ArgumentError(f"{name} must be Float32 (got {a.dtype})")
    if a.dim() < 1 or a.shape[0] != rows:
        raise _lib.DimensionMismatch(f"{name} must have size ({rows}, dims...), got {tuple(a.shape)}")
    if a.device.type != "cuda":
        a = a.to(device)
    rev = a.permute(*reversed(range(a.dim())))
    if not rev.is_contiguous():
        rev = rev.contiguous()
    return rev.reshape(-1), tuple(a.shape[1:]), was_numpy


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None and t.numel() > 0 else C.c_void_p(0)


def _stream(device):
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


# ---------------------------------------------------------------------------
# descriptor construction
# ---------------------------------------------------------------------------

def flatten_elements(elements) -> List[Tuple[int, object]]:
    """Flatten a chain into (element index, layer) pairs.

    CouplingBlocks give two layers with one element index (ldj_1 .+ ldj_2,
    src/Blocks.jl:136,149); a nested FlowChain is flattened into one element
    (its inner ldj is accumulated left to right, equal to the reference up to
    fp32 summation order when it contains blocks)."""
    from .chains import FlowChain

    out = []
    for e_idx, e in enumerate(elements):
        if isinstance(e, CouplingBlock):
            out += [(e_idx, e.layer_1), (e_idx, e.layer_2)]
        elif isinstance(e, FlowChain):
            for _, l in flatten_elements(e.layers):
                out.append((e_idx, l))
        elif isinstance(e, (RNVPCouplingLayer, NICECouplingLayer, NormalizationLayer)):
            out.append((e_idx, e))
        else:
            raise _lib.UnsupportedError(f"no fused kernel for flow element {type(e).__name__}")
    return out


def chain_dims(flat, n_hint: int | None = None) -> Tuple[int, int]:
    d = n = None
    for _, l in flat:
        if isinstance(l, NormalizationLayer):
            dd = l.x_min.shape[0]
            if d is not None and dd != d:
                raise _lib.DimensionMismatch("NormalizationLayer dimension does not match the chain")
            d = dd
        else:
            if d is not None and l.axes.d != d:
                raise _lib.DimensionMismatch("layers of a chain must share the dimension d")
            if n is not None and l.axes.n != n:
                raise _lib.DimensionMismatch("layers of a chain must share the number of conditions n")
            d, n = l.axes.d, l.axes.n
    if n is None:
        n = n_hint or 0
    return d, n


class _Desc:
    """Owns the ctypes descriptor and every host array it points to."""

    def __init__(self, flat, d, n):
        self.keep = []
        layers = (_lib.df_layer_desc * len(flat))()
        for i, (e_idx, l) in enumerate(flat):
            L = layers[i]
            L.element = e_idx
            if isinstance(l, NormalizationLayer):
                L.kind = _lib.DF_LAYER_NORM
                L.x_min = self._fp(l.x_min)
                L.x_max = self._fp(l.x_max)
                L.alpha = l.alpha
                L.beta = l.beta
                continue
            L.kind = _lib.DF_LAYER_RNVP if isinstance(l, RNVPCouplingLayer) else _lib.DF_LAYER_NICE
            L.n_af = len(l.axes.axis_af)
            L.axis_af = self._ip(l.axes.axis_af)
            L.n_nn = len(l.axes.axis_nn)
            L.axis_nn = self._ip(l.axes.axis_nn)
            if isinstance(l, RNVPCouplingLayer):
                L.n_dense_s, L.s_net = self._net(l.s_net)
            L.n_dense_t, L.t_net = self._net(l.t_net)
        self.keep.append(layers)
        self.desc = _lib.df_chain_desc(_lib.ABI_VERSION, d, n, len(flat), layers)

    def _fp(self, a):
        a = np.ascontiguousarray(a, dtype=np.float32)
        self.keep.append(a)
        return a.ctypes.data_as(C.POINTER(C.c_float))

    def _ip(self, a):
        a = np.ascontiguousarray(a, dtype=np.int32)
        self.keep.append(a)
        return a.ctypes.data_as(C.POINTER(C.c_int32))

    def _net(self, net):
        arr = (_lib.df_dense_desc * len(net))()
        for k, D in enumerate(net):
            W = np.asfortranarray(D.W, dtype=np.float32)  # Flux column-major (out, in)
            self.keep.append(W)
            arr[k].in_dim = D.in_dim
            arr[k].out_dim = D.out_dim
            arr[k].act = _lib.ACTIVATIONS[D.act]
            arr[k].W = W.ctypes.data_as(C.POINTER(C.c_float))
            arr[k].b = self._fp(D.b) if D.b is not None else C.POINTER(C.c_float)()
        self.keep.append(arr)
        return len(net), arr


def validate(elements, n_hint: int | None = None):
    """Host-only planning (no device): returns df_chain_info or raises."""
    lib = _lib.load()
    flat = flatten_elements(elements)
    d, n = chain_dims(flat, n_hint)
    desc = _Desc(flat, d, n)
    info = _lib.df_chain_info()
    _lib.check(lib.df_chain_validate(C.byref(desc.desc), C.byref(info)), "df_chain_validate")
    return info


class HIPChain:
    """A device-resident compiled chain (one ``df_chain`` handle per device)."""

    def __init__(self, elements, device=None, n_hint: int | None = None):
        torch = _torch()
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.HIPError("no HIP device visible: the fused kernels need an MI355X (gfx950)")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        flat = flatten_elements(elements)
        self.d, self.n = chain_dims(flat, n_hint)
        desc = _Desc(flat, self.d, self.n)
        h = C.c_void_p()
        _lib.check(self.lib.df_chain_create(C.byref(h), C.byref(desc.desc), self.device.index), "df_chain_create")
        self.handle = h
        self.info = _lib.df_chain_info()
        _lib.check(self.lib.df_chain_get_info(self.handle, C.byref(self.info)))
        self.bounds = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.df_chain_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None

    def set_weights(self, elements) -> None:
        """df_chain_set_weights: take the parameters of ``elements`` (same structure)."""
        flat = flatten_elements(elements)
        d, n = chain_dims(flat, self.n)
        if (d, n) != (self.d, self.n):
            raise _lib.DimensionMismatch("set_weights: (d, n) differ from the chain's")
        desc = _Desc(flat, d, n)
        _lib.check(self.lib.df_chain_set_weights(self.handle, C.byref(desc.desc)), "df_chain_set_weights")

    def set_theta_bounds(self, tmin, tmax):
        tmin = np.ascontiguousarray(tmin, dtype=np.float32).reshape(-1)
        tmax = np.ascontiguousarray(tmax, dtype=np.float32).reshape(-1)
        if tmin.shape[0] != self.n or tmax.shape[0] != self.n:
            raise _lib.DimensionMismatch("θ bounds must have n entries")
        _lib.check(self.lib.df_chain_set_theta_bounds(
            self.handle, tmin.ctypes.data_as(C.POINTER(C.c_float)), tmax.ctypes.data_as(C.POINTER(C.c_float))))
        self.bounds = (tmin.copy(), tmax.copy())

    # -- diagnostics ---------------------------------------------------------
    def clock_probe(self, on: bool = True) -> None:
        """df_chain_clock_probe: stamp the effective shader clock of later passes."""
        _lib.check(self.lib.df_chain_clock_probe(self.handle, 1 if on else 0), "df_chain_clock_probe")

    def clock_read(self):
        """df_chain_clock_read → (median GHz over workgroup slots, Σcycles/Σtime GHz, slots)."""
        med, mean, slots = C.c_double(), C.c_double(), C.c_int64()
        _lib.check(self.lib.df_chain_clock_read(self.handle, C.byref(med), C.byref(mean), C.byref(slots)),
                   "df_chain_clock_read")
        return med.value, mean.value, slots.value

    # -- raw entry points on flat device buffers ---------------------------
    def run(self, op: str, zbuf, thbuf, outbuf, ldjbuf, batch: int, flow: bool = False):
        fn = {
            ("forward", False): self.lib.df_chain_forward, ("forward", True): self.lib.df_flow_forward,
            ("backward", False): self.lib.df_chain_backward, ("backward", True): self.lib.df_flow_backward,
        }[(op, flow)]
        _lib.check(fn(self.handle, _ptr(zbuf), _ptr(thbuf), _ptr(outbuf), _ptr(ldjbuf), C.c_int64(batch),
                      _stream(self.device)), op)

    def run_inplace(self, zbuf, thbuf, batch: int, flow: bool = False):
        fn = self.lib.df_flow_forward_inplace if flow else self.lib.df_chain_forward_inplace
        _lib.check(fn(self.handle, _ptr(zbuf), _ptr(thbuf), C.c_int64(batch), _stream(self.device)), "forward!")

    def run_logpdf(self, xbuf, thbuf, lpbuf, batch: int):
        _lib.check(self.lib.df_flow_logpdf(self.handle, _ptr(xbuf), _ptr(thbuf), _ptr(lpbuf), C.c_int64(batch),
                                           _stream(self.device)), "logpdf")

    def run_logpdf_sum(self, xbuf, thbuf, sumbuf, batch: int):
        _lib.check(self.lib.df_flow_logpdf_sum(self.handle, _ptr(xbuf), _ptr(thbuf),
                                               C.c_void_p(sumbuf.data_ptr()), C.c_int64(batch),
                                               _stream(self.device)), "logpdf_sum")

    def run_sample(self, xbuf, thbuf, broadcast: bool, batch: int, seed: int, offset: int = 0):
        """df_flow_sample: device N(0, I) draw (Philox, seed/offset) + fused forward!."""
        _lib.check(self.lib.df_flow_sample(self.handle, _ptr(xbuf), _ptr(thbuf), 1 if broadcast else 0,
                                           C.c_int64(batch), C.c_uint64(seed), C.c_uint64(offset),
                                           _stream(self.device)), "sample")

    def random_normal(self, buf, count: int, seed: int, offset: int = 0):
        """df_random_normal: the draw df_flow_sample uses for the same (seed, offset)."""
        _lib.check(self.lib.df_random_normal(_ptr(buf), C.c_int64(count), C.c_uint64(seed), C.c_uint64(offset),
                                             _stream(self.device)), "random_normal")

    # -- array-level API ---------------------------------------------------
    def _inputs(self, y, theta, name):
        yb, dims, was_np = as_julia_device(y, self.d, self.device, name)
        batch = int(np.prod(dims)) if dims else 1
        thb = None
        if self.n > 0:
            if theta is None:
                raise _lib.DimensionMismatch("a conditional flow needs θ of size (n, dims...)")
            thb, tdims, _ = as_julia_device(theta, self.n, self.device, "θ")
            if tdims != dims:
                raise _lib.DimensionMismatch("x and θ must have the same size -- except for the first dimension")
        return yb, thb, dims, batch, was_np

    @staticmethod
    def _ldj_view(buf, dims):
        if not dims:
            return buf.reshape(())
        torch = _torch()
        rev = buf.reshape(tuple(reversed(dims)))
        return rev.permute(*reversed(range(len(dims))))

    def apply(self, op: str, y, theta=None, flow: bool = False):
        """forward / backward → (out, ldj) with the input's logical shape."""
        torch = _torch()
        yb, thb, dims, batch, was_np = self._inputs(y, theta, "input")
        outb, outv = julia_empty(self.d, dims, self.device)
        ldjb = torch.empty(batch, dtype=torch.float32, device=self.device)
        self.run(op, yb, thb, outb, ldjb, batch, flow)
        ldjv = self._ldj_view(ldjb, dims)
        if was_np:
            return _to_numpy(outv), _to_numpy(ldjv)
        return outv, ldjv

    def apply_inplace(self, z, theta=None, flow: bool = False):
        """forward! — mutates ``z`` (a column-major torch tensor) in place."""
        torch = _torch()
        if not isinstance(z, torch.Tensor) or z.device.type != "cuda":
            raise _lib.ArgumentError("forward! needs a device tensor (it mutates its argument)")
        zb, thb, dims, batch, _ = self._inputs(z, theta, "z")
        if zb.data_ptr() != z.data_ptr() or not z.permute(*reversed(range(z.dim()))).is_contiguous():
            raise _lib.ArgumentError("forward! needs z in Julia (column-major) memory order")
        self.run_inplace(zb, thb, batch, flow)
        return None

    def logpdf(self, x, theta=None):
        torch = _torch()
        xb, thb, dims, batch, was_np = self._inputs(x, theta, "x")
        lpb = torch.empty(batch, dtype=torch.float32, device=self.device)
        self.run_logpdf(xb, thb, lpb, batch)
        v = self._ldj_view(lpb, dims)
        return _to_numpy(v) if was_np else v

    def logpdf_sum(self, x, theta=None, out=None):
        torch = _torch()
        xb, thb, dims, batch, _ = self._inputs(x, theta, "x")
        s = out if out is not None else torch.empty(1, dtype=torch.float64, device=self.device)
        self.run_logpdf_sum(xb, thb, s, batch)
        return s, batch


def _to_numpy(t):
    return t.detach().cpu().numpy()
