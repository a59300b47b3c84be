"""densityflows.jl_amd — MI355X-native (gfx950) hot path of DensityFlows.jl.

The Python host side mirrors the reference's Julia API (FlowChain,
CouplingLayer, CouplingBlock, NormalizationLayer, Flow, forward / backward /
forward!, logpdf, sample); every evaluation runs in the fused HIP kernels of
``libdensityflows_hip.so`` through its C ABI (include/densityflows_hip.h).

Import as ``densityflows_amd`` (a symlink to this directory at the repo root).
"""
from . import _lib
from ._lib import (ArgumentError, DimensionMismatch, HIPError, HIPLibraryError, UnsupportedError)
from .axes import CouplingAxes, is_reverse, reverse
from .chains import FlowChain, backward, concatenate, forward, forward_, forward_inplace
from .data import (DataArrays, DataPartition, MetaData, dflt_theta, maximum_theta, minimum_theta,
                   normalize_input, resize_output)
from .flows import (Flow, MvNormal, logpdf, nll_partial_sum, pdf, predict, sample, training_loss,
                    validation_loss)
from .layers import (Chain, CouplingBlock, CouplingLayer, Dense, FlowElement, NICECouplingLayer,
                     NormalizationLayer, RNVPCouplingLayer, default_net)
from .train import Adam, TrainState, load_trainables, setup, train_, trainables

__version__ = "0.1.0"


def summarize(obj) -> str:
    """``summarize`` / ``@summary`` — returns the text the reference prints."""
    return obj.summarize()


def library_path() -> str:
    return _lib.LIB_PATH


def load_library():
    """Load the native library (raises HIPLibraryError if it was not built)."""
    return _lib.load()
