"""Test helpers for user-defined ops: builds tests/user_ops.c (host
MPI_User_functions) and, on a GPU box, tests/user_ops_dev.hip (the same ops
as stream-ordered device functions)."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# name -> (datatype handle, commute flag the tests create it with, numpy dtype)
UOPS = {
    "addem": (6, 1, np.int32),
    "assoc": (6, 0, np.int32),
    "add_f64": (11, 1, np.float64),
    "fsum": (10, 1, np.float32),
    "mix": (7, 0, np.uint32),
    "affine": (9, 0, np.uint64),
}

_host = None
_dev = None


def _build(src, out, cmd):
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        subprocess.check_call(cmd)
    return out


def host_lib():
    """The host MPI_User_function library (gcc, built once per session)."""
    global _host
    if _host is None:
        d = tempfile.mkdtemp(prefix="mvx_uops_")
        so = os.path.join(d, "libuops.so")
        _build(os.path.join(HERE, "user_ops.c"), so,
               ["gcc", "-O2", "-std=gnu99", "-shared", "-fPIC", os.path.join(HERE, "user_ops.c"), "-o", so])
        _host = ctypes.CDLL(so)
    return _host


def host_fn(name):
    """Address of uop_<name> (a C MPI_User_function)."""
    return ctypes.cast(getattr(host_lib(), "uop_" + name), ctypes.c_void_p).value


def dev_lib():
    """The device-op library (hipcc for gfx950, built once per session)."""
    global _dev
    if _dev is None:
        d = tempfile.mkdtemp(prefix="mvx_duops_")
        so = os.path.join(d, "libduops.so")
        src = os.path.join(HERE, "user_ops_dev.hip")
        _build(src, so, ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                         "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero", src, "-o", so])
        _dev = ctypes.CDLL(so)
    return _dev


def dev_fn(name):
    return ctypes.cast(getattr(dev_lib(), "duop_" + name), ctypes.c_void_p).value


def rand_for(name, n, seed):
    rng = np.random.default_rng(seed)
    dt = UOPS[name][2]
    if name in ("addem", "assoc"):
        return rng.integers(-1000, 1000, n).astype(dt)
    if name == "add_f64":
        return (rng.standard_normal(n) * 10.0 ** rng.integers(-3, 3, n)).astype(dt)
    if name == "fsum":
        return (rng.standard_normal(n) * 10.0 ** rng.integers(-4, 4, n)).astype(dt)
    if name == "mix":
        return rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(dt)
    return rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
