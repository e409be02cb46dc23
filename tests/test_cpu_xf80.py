"""CPU: the device's x87 long double emulation against the host x87.

mvapich-cce_amd/csrc/mvx_xf80.h is the arithmetic the MPI_LONG_DOUBLE and
MPI_LONG_DOUBLE_INT kernels run.  Compiled for the host (tests/xf80_host.cc),
it must produce the same 16 bytes per element (value and untouched slot
padding) as the oracle's `long double` ops, which this container's x87 unit
evaluates exactly as the reference's global_ops.c does, over every operand
class (tests/mvxtest.py xf_patterns).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import mvxtest as T

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def xf_host(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("xf80") / "libxf80_host.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I",
                           os.path.join(ROOT, "mvapich-cce_amd", "csrc"),
                           os.path.join(HERE, "xf80_host.cc"), "-o", so])
    L = ctypes.CDLL(so)
    L.xf_host_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    return L


def _first_diff(got, ref, b, a):
    g, r = got.view(np.uint8).reshape(got.size, -1), ref.view(np.uint8).reshape(ref.size, -1)
    bad = np.nonzero((g != r).any(1))[0]
    if not bad.size:
        return None
    i = bad[0]
    return "%d/%d elements differ; first %d: in %s inout %s -> got %s ref %s" % (
        bad.size, got.size, i, b.view(np.uint8).reshape(b.size, -1)[i].tobytes().hex(),
        a.view(np.uint8).reshape(a.size, -1)[i].tobytes().hex(), g[i].tobytes().hex(), r[i].tobytes().hex())


@pytest.mark.parametrize("op", [100, 101, 102, 103, 104, 106, 108])
def test_long_double_ops_match_x87(oracle, xf_host, op):
    n = 400000
    for seed in (1, 2):
        b, a = T.xf_operands(n, seed + op)
        ref, got = T.clone(a), T.clone(a)
        assert oracle.op(op, 12, b.view(np.uint8), ref.view(np.uint8), n) == 0
        assert xf_host.xf_host_op(op, 12, b.ctypes.data, got.ctypes.data, n) == 0
        msg = _first_diff(got, ref, b, a)
        assert msg is None, msg


@pytest.mark.parametrize("op", [110, 111])
def test_long_double_int_loc_match_x87(oracle, xf_host, op):
    n = 200000
    b, a = T.xfi_operands(n, op)
    ref, got = T.clone(a), T.clone(a)
    assert oracle.op(op, 22, b.view(np.uint8), ref.view(np.uint8), n) == 0
    assert xf_host.xf_host_op(op, 22, b.ctypes.data, got.ctypes.data, n) == 0
    msg = _first_diff(got, ref, b, a)
    assert msg is None, msg


def test_pattern_classes_present():
    """The generator reaches every class the emulation branches on."""
    b, a = T.xf_operands(100000, 3)
    e = a["se"] & 0x7fff
    j = a["m"] >> np.uint64(63)
    assert ((e == 0) & (j == 1)).any() and ((e == 0) & (j == 0) & (a["m"] != 0)).any()    # pseudo-/denormals
    assert ((e > 0) & (e < 0x7fff) & (j == 0)).any()                                     # unnormals
    assert ((e == 0x7fff) & (j == 0)).any()                                              # pseudo-inf/NaN
    assert ((e == 0x7fff) & (a["m"] == np.uint64(1 << 63))).any()                        # infinity


def test_add_normal_operands_every_exponent_gap(oracle, xf_host):
    """The 64-bit fast path of xf::add (normal operands, exponent gap <= 64)
    against the x87: every gap 0..80 (beyond 64 the general path), both
    signs, exponents at the denormal and overflow edges, significands with
    long runs of ones / zeros (carries, borrows, ties at the rounding bit)."""
    rng = np.random.default_rng(7)
    n = 200000
    dt = np.dtype([("m", "<u8"), ("se", "<u2"), ("p0", "<u2"), ("p1", "<u4")])
    a = np.zeros(n, dt)
    b = np.zeros(n, dt)
    gap = rng.integers(0, 81, n)
    base = rng.choice(np.array([1, 2, 3, 64, 65, 66, 100, 16383, 0x7ffe - 80, 0x7ffd, 0x7ffe]), n)
    ea = np.clip(base + rng.integers(0, 3, n), 1, 0x7ffe)
    eb = np.clip(ea - gap, 1, 0x7ffe)
    swap = rng.random(n) < 0.5
    ea, eb = np.where(swap, eb, ea), np.where(swap, ea, eb)
    def sig(k):
        m = rng.integers(0, 1 << 63, k, dtype=np.uint64) | np.uint64(1 << 63)
        pick = rng.integers(0, 4, k)
        m = np.where(pick == 0, np.uint64(0xFFFFFFFFFFFFFFFF), m)                  # all ones
        m = np.where(pick == 1, np.uint64(1 << 63) | rng.integers(0, 4, k, dtype=np.uint64), m)
        return m
    a["m"], b["m"] = sig(n), sig(n)
    a["se"] = (ea | (rng.integers(0, 2, n) << 15)).astype(np.uint16)
    b["se"] = (eb | (rng.integers(0, 2, n) << 15)).astype(np.uint16)
    a["p0"], a["p1"] = 0x1234, 0x89abcdef
    ref, got = a.copy(), a.copy()
    assert oracle.op(102, 12, b.view(np.uint8), ref.view(np.uint8), n) == 0
    assert xf_host.xf_host_op(102, 12, b.ctypes.data, got.ctypes.data, n) == 0
    msg = _first_diff(got, ref, b, a)
    assert msg is None, msg
