"""ctypes binding of ``libdensityflows_hip.so`` (include/densityflows_hip.h).

The shared library is built in-tree (``__graft_entry__.build()`` /
``make -C densityflows.jl_amd/csrc``).  There is no CPU fallback: if the
library is missing every entry point raises ``HIPLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdensityflows_hip.so")

ABI_VERSION = 4

# df_status
DF_OK = 0
DF_ERR_INVALID = -1
DF_ERR_SHAPE = -2
DF_ERR_HIP = -3
DF_ERR_UNSUPPORTED = -4
DF_ERR_NOMEM = -5
DF_ERR_NONFINITE = -6

# df_dtype
DF_DTYPE_F32 = 0
DF_DTYPE_F64 = 1
DF_COMM_ID_BYTES = 128

# df_theta_input (df_train_set_theta_input)
DF_THETA_AUTO = 0
DF_THETA_RAW = 1
DF_THETA_GIVEN = 2

# df_layer_kind
DF_LAYER_RNVP = 0
DF_LAYER_NICE = 1
DF_LAYER_NORM = 2

# df_act
ACTIVATIONS = {
    "identity": 0, "relu": 1, "tanh": 2, "sigmoid": 3, "softplus": 4,
    "logcosh": 5, "leakyrelu": 6, "elu": 7, "swish": 8,
}


class HIPLibraryError(RuntimeError):
    """The native library could not be loaded (no CPU fallback exists)."""


class ArgumentError(ValueError):
    """Mirror of Julia's ArgumentError (invalid structure / argument)."""


class DimensionMismatch(AssertionError):
    """Mirror of the reference's @assert / DimensionMismatch shape errors."""


class UnsupportedError(NotImplementedError):
    """Structure outside the fused kernels' limits (see df_limits)."""


class HIPError(RuntimeError):
    """HIP runtime failure inside the library."""


class NonFiniteError(ValueError):
    """DF_ERR_NONFINITE: train!(...; debug=true) found a NaN/Inf loss
    (src/Flows.jl:404-409 throws an ArgumentError there)."""


class df_dense_desc(C.Structure):
    _fields_ = [("in_dim", C.c_int32), ("out_dim", C.c_int32), ("act", C.c_int32),
                ("W", C.POINTER(C.c_float)), ("b", C.POINTER(C.c_float))]


class df_layer_desc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("element", C.c_int32),
                ("n_af", C.c_int32), ("axis_af", C.POINTER(C.c_int32)),
                ("n_nn", C.c_int32), ("axis_nn", C.POINTER(C.c_int32)),
                ("n_dense_s", C.c_int32), ("s_net", C.POINTER(df_dense_desc)),
                ("n_dense_t", C.c_int32), ("t_net", C.POINTER(df_dense_desc)),
                ("x_min", C.POINTER(C.c_float)), ("x_max", C.POINTER(C.c_float)),
                ("alpha", C.c_float), ("beta", C.c_float)]


class df_chain_desc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("d", C.c_int32), ("n", C.c_int32),
                ("n_layers", C.c_int32), ("layers", C.POINTER(df_layer_desc))]


class df_limits(C.Structure):
    _fields_ = [("max_state", C.c_int32), ("max_hidden", C.c_int32),
                ("max_af", C.c_int32), ("max_layers", C.c_int32)]


class df_chain_info(C.Structure):
    _fields_ = [("d", C.c_int32), ("n", C.c_int32), ("n_layers", C.c_int32),
                ("hidden_tiles", C.c_int32), ("samples_per_block", C.c_int32),
                ("n_stages", C.c_int32), ("n_params", C.c_int64),
                ("flops_per_sample", C.c_double), ("weight_bytes", C.c_int64),
                ("kernel", C.c_int32), ("reserved", C.c_int32), ("split_flops_per_sample", C.c_double)]


class df_adam(C.Structure):
    _fields_ = [("eta", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("epsilon", C.c_float)]


_FP = C.POINTER(C.c_float)
_VP = C.c_void_p
_I64 = C.c_int64

# name -> (restype, argtypes); every symbol include/densityflows_hip.h declares
SIGNATURES = {
    "df_get_abi_version": (C.c_int, []),
    "df_last_error": (C.c_char_p, []),
    "df_get_limits": (C.c_int, [C.POINTER(df_limits)]),
    "df_chain_validate": (C.c_int, [C.POINTER(df_chain_desc), C.POINTER(df_chain_info)]),
    "df_chain_create": (C.c_int, [C.POINTER(_VP), C.POINTER(df_chain_desc), C.c_int]),
    "df_chain_destroy": (C.c_int, [_VP]),
    "df_chain_get_info": (C.c_int, [_VP, C.POINTER(df_chain_info)]),
    "df_chain_set_theta_bounds": (C.c_int, [_VP, _FP, _FP]),
    "df_chain_forward": (C.c_int, [_VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    "df_chain_backward": (C.c_int, [_VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    "df_chain_forward_inplace": (C.c_int, [_VP, _VP, _VP, _I64, _VP]),
    "df_flow_forward": (C.c_int, [_VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    "df_flow_backward": (C.c_int, [_VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    "df_flow_forward_inplace": (C.c_int, [_VP, _VP, _VP, _I64, _VP]),
    "df_flow_logpdf": (C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP]),
    "df_flow_logpdf_sum": (C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP]),
    "df_chain_logpdf": (C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP]),
    "df_chain_logpdf_sum": (C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP]),
    "df_train_create": (C.c_int, [C.POINTER(_VP), _VP, C.POINTER(df_adam)]),
    "df_train_destroy": (C.c_int, [_VP]),
    "df_train_create_ex": (C.c_int, [C.POINTER(_VP), _VP, C.POINTER(df_adam), C.c_int]),
    "df_train_sweep": (C.c_int, [_VP, C.POINTER(C.c_int)]),
    "df_train_num_params": (C.c_int, [_VP, C.POINTER(_I64)]),
    "df_train_gradient": (C.c_int, [_VP, _VP, _VP, _I64, _I64, _VP, _VP]),
    "df_train_grad_ptr": (C.c_int, [_VP, C.POINTER(_VP)]),
    "df_train_apply": (C.c_int, [_VP, _VP]),
    "df_train_step": (C.c_int, [_VP, _VP, _VP, _I64, _VP, _VP]),
    "df_train_step_graph": (C.c_int, [_VP, _VP, _VP, _I64, _I64, _VP, _VP]),
    "df_train_get_params": (C.c_int, [_VP, _FP, _I64]),
    "df_train_set_params": (C.c_int, [_VP, _FP, _I64]),
    "df_train_set_debug": (C.c_int, [_VP, C.c_int]),
    "df_train_set_theta_input": (C.c_int, [_VP, C.c_int]),
    "df_chain_set_weights": (C.c_int, [_VP, C.POINTER(df_chain_desc)]),
    "df_comm_get_unique_id": (C.c_int, [_VP]),
    "df_comm_init_rank": (C.c_int, [C.POINTER(_VP), C.c_int, _VP, C.c_int, C.c_int]),
    "df_comm_destroy": (C.c_int, [_VP]),
    "df_comm_get_info": (C.c_int, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "df_comm_allreduce_sum": (C.c_int, [_VP, _VP, _I64, C.c_int, _VP]),
    "df_flow_nll": (C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP, _VP]),
    "df_chain_nll": (C.c_int, [_VP, _VP, _VP, _VP, _I64, _VP, _VP]),
    "df_train_allreduce_gradient": (C.c_int, [_VP, _VP, _VP]),
    "df_train_step_dist": (C.c_int, [_VP, _VP, _VP, _VP, _I64, _I64, _VP, _VP]),
    "df_flow_sample": (C.c_int, [_VP, _VP, _VP, C.c_int, _I64, C.c_uint64, C.c_uint64, _VP]),
    "df_random_normal": (C.c_int, [_VP, _I64, C.c_uint64, C.c_uint64, _VP]),
    "df_chain_clock_probe": (C.c_int, [_VP, C.c_int]),
    "df_chain_clock_read": (C.c_int, [_VP, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(_I64)]),
    "df_device_alloc": (C.c_int, [C.POINTER(_VP), C.c_size_t]),
    "df_device_free": (C.c_int, [_VP]),
    "df_memcpy_h2d": (C.c_int, [_VP, _VP, C.c_size_t, _VP]),
    "df_memcpy_d2h": (C.c_int, [_VP, _VP, C.c_size_t, _VP]),
    "df_stream_synchronize": (C.c_int, [_VP]),
}

_lock = threading.Lock()
_lib = None


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raise HIPLibraryError if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("DENSITYFLOWS_HIP_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise HIPLibraryError(
                f"{p} not found: build it with __graft_entry__.build() or "
                "`make -C densityflows.jl_amd/csrc` (there is no CPU fallback)")
        try:
            lib = C.CDLL(p)
        except OSError as e:  # pragma: no cover - depends on the host
            raise HIPLibraryError(f"cannot load {p}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            # a symbol an older build lacks (A/B runs against a saved library) stays
            # unbound: calling it raises AttributeError; tests/test_host.py checks that the
            # in-tree build exports every one
            try:
                fn = getattr(lib, name)
            except AttributeError:
                continue
            fn.restype = res
            fn.argtypes = args
        if lib.df_get_abi_version() != ABI_VERSION:
            raise HIPLibraryError("ABI version mismatch between the Python mirror and the library")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str = ""):
    """Map a df_status to the reference's exception types."""
    if rc == DF_OK:
        return
    msg = load().df_last_error().decode("utf-8", "replace")
    if what:
        msg = f"{what}: {msg}"
    if rc == DF_ERR_INVALID:
        raise ArgumentError(msg)
    if rc == DF_ERR_SHAPE:
        raise DimensionMismatch(msg)
    if rc == DF_ERR_UNSUPPORTED:
        raise UnsupportedError(msg)
    if rc == DF_ERR_NOMEM:
        raise MemoryError(msg)
    if rc == DF_ERR_NONFINITE:
        raise NonFiniteError(msg)
    raise HIPError(f"[{rc}] {msg}")
