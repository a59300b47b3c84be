"""Convert the reference's test fixture ``test/datatest.jld2`` into .npy files.

Run ONLY in the build container (the reference tree does not exist on the GPU
box).  JLD2 files are HDF5-compatible; the HDF5 command-line tool ``h5dump``
dumps each dataset as raw little-endian float32 (no code from the file is
executed).  Datasets (Julia shapes): ``x`` 5×1000 Float32, ``θ`` 1×1000
Float32 (values {-1, 2}, 500 each) — used by test/runtests.jl:97-121.

Outputs (logical Julia shape, C-contiguous numpy arrays):
    tests/golden/datatest_x.npy      (5, 1000) float32
    tests/golden/datatest_theta.npy  (1, 1000) float32
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference/test/datatest.jld2"
H5DUMP = "/opt/conda/bin/h5dump"
HERE = os.path.dirname(os.path.abspath(__file__))


def dump(name, count):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "d.bin")
        subprocess.run([H5DUMP, "-d", name, "-b", "LE", "-o", out, REF],
                       check=True, stdout=subprocess.DEVNULL)
        a = np.fromfile(out, dtype="<f4")
    assert a.size == count, (name, a.size)
    return a


def main():
    if not os.path.exists(REF):
        print("reference fixture not present; nothing to do", file=sys.stderr)
        return 1
    # On disk the HDF5 dataspace is (1000, 5) row-major == Julia 5×1000
    # column-major: sample j's 5 values are contiguous.
    x = dump("x", 5000).reshape(1000, 5).T.copy()
    th = dump("θ", 1000).reshape(1000, 1).T.copy()
    np.save(os.path.join(HERE, "datatest_x.npy"), x)
    np.save(os.path.join(HERE, "datatest_theta.npy"), th)
    print("x", x.shape, x.mean(axis=1), "theta", th.shape, np.unique(th, return_counts=True))
    return 0


if __name__ == "__main__":
    sys.exit(main())
