"""Shared helpers of the test suite (inputs, device transfer, comparisons)."""
import numpy as np

MPI_FLOAT, MPI_DOUBLE = 10, 11
PAIRS = (17, 18, 19, 20, 21)
ALL_OPS = list(range(100, 112))
# every handle the device path knows, plus one unregistered-on-device (BYTE is
# only valid for B* ops) and the two x87 long double types
ALL_TYPES = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 17, 18, 19, 20, 21, 22, 23, 24]

_np_cache = {}


def np_dtype(dtype):
    import importlib
    mvx = importlib.import_module("mvapich-cce_amd")
    if dtype == 12:
        return np.dtype(np.longdouble)
    if dtype == 22:
        return np.dtype({"names": ["v", "l"], "formats": [np.longdouble, np.int32], "offsets": [0, 16],
                         "itemsize": 32})
    return mvx.NP_DTYPE[dtype]


def rand_vec(dtype, n, seed):
    """Random elements with plenty of ties, signs, zeros and (for floats)
    the odd special value, so every branch of every op is exercised."""
    rng = np.random.default_rng(seed)
    dt = np_dtype(dtype)
    if dt.names:
        out = np.zeros(n, dt)
        vt = dt.fields["v"][0]
        out["v"] = _rand_scalar(vt, n, rng)
        out["l"] = rng.integers(-5, 50, n)
        return out
    if dt.kind == "c":
        ft = np.float32 if dt.itemsize == 8 else np.float64
        re = _rand_scalar(np.dtype(ft), n, rng)
        im = _rand_scalar(np.dtype(ft), n, rng)
        return (re + 1j * im).astype(dt)
    return _rand_scalar(dt, n, rng)


def _rand_scalar(dt, n, rng):
    if dt.kind == "f":
        if dt == np.longdouble:
            return rng.integers(-9, 9, n).astype(np.longdouble)
        v = rng.standard_normal(n) * np.exp2(rng.integers(-20, 20, n))
        v = np.where(rng.random(n) < 0.25, rng.integers(-3, 4, n), v)   # ties and zeros
        v = v.astype(dt)
        sp = rng.random(n)
        v[sp < 0.01] = np.nan
        v[(sp >= 0.01) & (sp < 0.015)] = np.inf
        v[(sp >= 0.015) & (sp < 0.02)] = -0.0
        return v
    info = np.iinfo(dt)
    wide = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    small = rng.integers(-3 if info.min < 0 else 0, 4, n).astype(dt)
    return np.where(rng.random(n) < 0.3, small, wide).astype(dt)


def clone(a):
    """Byte-exact copy (ndarray.copy() skips the padding of structured dtypes)."""
    a = np.ascontiguousarray(a)
    return a.view(np.uint8).copy().view(a.dtype)


def to_dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to("cuda")


def from_dev(t, like=None):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def bytes_equal(got_u8, ref):
    return np.array_equal(np.asarray(got_u8).view(np.uint8), np.ascontiguousarray(ref).view(np.uint8))


def oracle_rc(O, op, dtype):
    a = np.zeros(64, np.uint8)
    b = np.zeros(64, np.uint8)
    return O.op(op, dtype, a, b, 1)


def _float_parts(arr):
    """(bits, isnan) over every float lane of an element array."""
    a = np.ascontiguousarray(arr)
    dt = a.dtype
    if dt.names:
        v = a["v"]
        if v.dtype.kind != "f":
            return None
        return v.view(np.uint32 if v.dtype.itemsize == 4 else np.uint64), np.isnan(v)
    if dt.kind == "c":
        f = a.view(np.float32 if dt.itemsize == 8 else np.float64)
        return f.view(np.uint32 if f.dtype.itemsize == 4 else np.uint64), np.isnan(f)
    if dt.kind == "f":
        return a.view(np.uint32 if dt.itemsize == 4 else np.uint64), np.isnan(a)
    return None


def assert_same(op, dtype, got_u8, ref, typemap_only=False):
    """Bit-exact, except: NaN results of SUM/PROD need only both be NaN."""
    ref = np.ascontiguousarray(ref)
    got = np.asarray(got_u8).view(np.uint8)[: ref.nbytes].view(ref.dtype)
    if ref.dtype.names and typemap_only:
        assert np.array_equal(got["l"], ref["l"]), "loc differs"
        gv, rv = np.ascontiguousarray(got["v"]), np.ascontiguousarray(ref["v"])
        if op in (102, 103) and gv.dtype.kind == "f":
            ok = (gv.view(np.uint8) == rv.view(np.uint8)).reshape(gv.size, -1).all(1) | (np.isnan(gv) & np.isnan(rv))
            assert ok.all(), "value bits differ"
        else:
            assert np.array_equal(gv.view(np.uint8), rv.view(np.uint8)), "value bits differ"
        return
    if op in (102, 103):
        fp = _float_parts(ref)
        if fp is not None:
            gbits, gnan = _float_parts(got)
            rbits, rnan = fp
            assert np.array_equal(gnan, rnan), "NaN positions differ"
            ok = (gbits == rbits) | (gnan & rnan)
            bad = np.nonzero(~ok)[0]
            assert bad.size == 0, "%d lanes differ, first %s: got %x ref %x" % (
                bad.size, bad[:5], gbits[bad[0]], rbits[bad[0]])
            if ref.dtype.names:
                assert np.array_equal(got["l"], ref["l"])
            return
    gb, rb = got.view(np.uint8), ref.view(np.uint8)
    if not np.array_equal(gb, rb):
        diff = np.nonzero(gb != rb)[0]
        raise AssertionError("%d bytes differ, first at byte %d (elem %d): got %s ref %s" % (
            diff.size, diff[0], diff[0] // ref.dtype.itemsize, got[diff[0] // ref.dtype.itemsize],
            ref[diff[0] // ref.dtype.itemsize]))
