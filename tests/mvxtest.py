"""Shared helpers of the test suite (inputs, device transfer, comparisons)."""
import numpy as np

MPI_FLOAT, MPI_DOUBLE = 10, 11
PAIRS = (17, 18, 19, 20, 21, 22, 29, 32, 33)
ALL_OPS = list(range(100, 112))
# every handle the device path knows, plus one unregistered-on-device (BYTE is
# only valid for B* ops) and the two x87 long double types
# and the Fortran types 25-33
ALL_TYPES = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 17, 18, 19, 20, 21, 22, 23, 24,
             25, 26, 27, 28, 29, 30, 31, 32, 33]

_np_cache = {}


def np_dtype(dtype):
    import importlib
    mvx = importlib.import_module("mvapich-cce_amd")
    return mvx.NP_DTYPE[dtype]


def rand_vec(dtype, n, seed):
    """Random elements with plenty of ties, signs, zeros and (for floats)
    the odd special value, so every branch of every op is exercised."""
    rng = np.random.default_rng(seed)
    dt = np_dtype(dtype)
    if dtype == 12:
        return xf_rand(n, rng).view(np.longdouble)
    if dtype == 25:     # MPI_LOGICAL: .TRUE. (1), .FALSE. (0) and other words
        return rng.choice(np.array([0, 1, 1, 0, 2, -1, 1, 0], np.int32), n)
    if dtype == 22:
        out = np.zeros(n, dt)
        u = out.view(np.uint8).reshape(n, 32)
        u[:, :16] = xf_rand(n, rng).view(np.uint8).reshape(n, 16)
        u[:, 20:] = rng.integers(0, 256, (n, 12), dtype=np.uint8)
        out["l"] = rng.integers(-5, 50, n)
        return out
    if dt.names:
        out = np.zeros(n, dt)
        vt = dt.fields["v"][0]
        out["v"] = _rand_scalar(vt, n, rng)
        out["l"] = rng.integers(-5, 50, n)
        return out
    return _rand_scalar(dt, n, rng)


def _rand_scalar(dt, n, rng):
    if dt.kind == "c":
        # lane-wise: `re + 1j*im` would turn an inf / NaN imaginary draw into
        # a NaN real lane too (1j*inf = nan+infj), so special values land
        # only in the lane they were drawn for
        ft = np.dtype(np.float32 if dt.itemsize == 8 else np.float64)
        out = np.empty(n, dt)
        lanes = out.view(ft)
        lanes[0::2] = _rand_scalar(ft, n, rng)
        lanes[1::2] = _rand_scalar(ft, n, rng)
        return out
    if dt.kind == "f":
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
    """Bit-exact, except: NaN results of SUM/PROD need only both be NaN
    (f32/f64; the x87 types are emulated exactly, NaN payloads included)."""
    ref = np.ascontiguousarray(ref)
    got = np.asarray(got_u8).view(np.uint8)[: ref.nbytes].view(ref.dtype)
    if dtype in (12, 22):
        w = ref.dtype.itemsize
        keep = 20 if (dtype == 22 and typemap_only) else w      # type map: value slot + loc
        gb = got.view(np.uint8).reshape(-1, w)[:, :keep]
        rb = ref.view(np.uint8).reshape(-1, w)[:, :keep]
        bad = np.nonzero((gb != rb).any(1))[0]
        assert bad.size == 0, "%d x87 elements differ, first %d: got %s ref %s" % (
            bad.size, bad[0], gb[bad[0]].tobytes().hex(), rb[bad[0]].tobytes().hex())
        return
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


# ---------------------------------------------------------------------------
# x87 long double bit patterns (MPI_LONG_DOUBLE = 12, MPI_LONG_DOUBLE_INT = 22)

XF_DT = np.dtype({"names": ["m", "se", "pad0", "pad1"], "formats": [np.uint64, np.uint16, np.uint16, np.uint32],
                  "offsets": [0, 8, 10, 12], "itemsize": 16})
XFI_DT = np.dtype({"names": ["m", "se", "pad0", "pad1", "l", "pa", "pb", "pc"],
                   "formats": [np.uint64, np.uint16, np.uint16, np.uint32, np.int32, np.int32, np.int32, np.int32],
                   "offsets": [0, 8, 10, 12, 16, 20, 24, 28], "itemsize": 32})


def xf_patterns(n, rng):
    """x87 extended bit patterns covering every operand class the x87 unit
    distinguishes: normals near 1 (so sums interact and cancel), the whole
    exponent range, products that underflow to denormals or overflow,
    denormals, pseudo-denormals, zeros, infinities, quiet and signalling
    NaNs, the real indefinite, unnormals, pseudo-infinities and pseudo-NaNs.
    Slot padding is random, to check it is carried from the inout operand."""
    J = np.uint64(1 << 63)
    m = rng.integers(0, 1 << 63, n, dtype=np.uint64, endpoint=False) * np.uint64(2) + \
        rng.integers(0, 2, n, dtype=np.uint64)
    sign = rng.integers(0, 2, n).astype(np.uint32) << 15
    cls = rng.integers(0, 100, n)
    e = np.empty(n, np.int64)
    near = cls < 40
    e[near] = 16383 + rng.integers(-66, 67, near.sum())
    wide = (cls >= 40) & (cls < 50)
    e[wide] = rng.integers(1, 0x7fff, wide.sum())
    lo = (cls >= 50) & (cls < 60)             # products near the underflow edge
    e[lo] = 8192 + rng.integers(-40, 40, lo.sum())
    hi = (cls >= 60) & (cls < 65)             # products near overflow
    e[hi] = 24575 + rng.integers(-3, 3, hi.sum())
    tiny = (cls >= 65) & (cls < 75)           # denormals and the bottom binades
    e[tiny] = rng.integers(0, 3, tiny.sum())
    small_int = (cls >= 75) & (cls < 82)      # exact small integers: ties, zeros, cancellation
    ints = rng.integers(-4, 5, n)
    spec = cls >= 82
    e[spec] = 0
    mm = m | J
    # denormals (J = 0) at exponent 0 two times in three, pseudo-denormals otherwise
    den = tiny & (e == 0)
    mm = np.where(den & (rng.random(n) < 0.67), m & ~J, mm)
    se = (sign | e.astype(np.uint32)).astype(np.uint32)
    # small integers
    k = np.abs(ints).astype(np.uint64)
    kk = np.maximum(k, 1)
    lz = np.array([64 - int(v).bit_length() for v in kk], np.uint64)
    mi = np.where(k == 0, np.uint64(0), kk << lz)
    ei = np.where(k == 0, 0, 16383 + 63 - lz.astype(np.int64))
    si = np.where(ints < 0, 1 << 15, 0)
    mm = np.where(small_int, mi, mm)
    se = np.where(small_int, si | ei, se)
    # specials
    sk = rng.integers(0, 10, n)
    frac = m & np.uint64((1 << 62) - 1)
    frac = np.where(frac == 0, np.uint64(1), frac)
    specials = [
        (np.uint64(0), 0),                          # zero
        (J, 0x7fff),                                # infinity
        (J | np.uint64(1 << 62) | (frac & np.uint64(0xff)), 0x7fff),   # QNaN, small payloads (ties)
        (J | np.uint64(1 << 62) | frac, 0x7fff),    # QNaN
        (J | frac, 0x7fff),                         # SNaN
        (np.uint64(0xC000000000000000), 0x7fff),    # indefinite (with sign: either)
        (m & ~J, None),                             # unnormal (random exponent)
        (np.uint64(0), 0x7fff),                     # pseudo-infinity
        (frac, 0x7fff),                             # pseudo-NaN
        (J | (frac & np.uint64(0xff)), 0x7fff),     # SNaN, small payloads
    ]
    rnd_e = rng.integers(1, 0x7fff, n)
    for i, (mv, ev) in enumerate(specials):
        sel = spec & (sk == i)
        mv = np.broadcast_to(np.asarray(mv, np.uint64), (n,))
        ev = rnd_e if ev is None else np.full(n, ev)
        mm = np.where(sel, mv, mm)
        se = np.where(sel, sign | ev, se)
    out = np.zeros(n, XF_DT)
    out["m"] = mm
    out["se"] = se.astype(np.uint16)
    out["pad0"] = rng.integers(0, 1 << 16, n, dtype=np.uint16)
    out["pad1"] = rng.integers(0, 1 << 32, n, dtype=np.uint32)
    return out


def xf_rand(n, rng):
    """Mostly finite values near 1 (so the association of a sum or product
    shows in the rounding), with one element in five from xf_patterns."""
    out = xf_patterns(n, rng)
    near = rng.random(n) < 0.8
    m = rng.integers(0, 1 << 63, n, dtype=np.uint64) | np.uint64(1 << 63)
    se = (16383 + rng.integers(-8, 9, n)) | (rng.integers(0, 2, n) << 15)
    out["m"] = np.where(near, m, out["m"])
    out["se"] = np.where(near, se, out["se"]).astype(np.uint16)
    return out


def xf_operands(n, seed):
    """(in, inout) operand pairs: independent patterns, plus b related to a
    (negated, equal, nearby, or an exact half-ulp below it) often enough to
    hit cancellation, ties to even, NaN significand ties and equal values."""
    rng = np.random.default_rng(seed)
    a = xf_patterns(n, rng)
    b = xf_patterns(n, rng)
    rel = rng.integers(0, 10, n)
    sel = rel == 0                                  # -a
    b["m"][sel] = a["m"][sel]
    b["se"][sel] = a["se"][sel] ^ np.uint16(0x8000)
    sel = rel == 1                                  # a
    b["m"][sel] = a["m"][sel]
    b["se"][sel] = a["se"][sel]
    sel = rel == 2                                  # -a, low bits perturbed
    b["m"][sel] = a["m"][sel] ^ rng.integers(0, 1 << 8, sel.sum(), dtype=np.uint64)
    b["se"][sel] = a["se"][sel] ^ np.uint16(0x8000)
    sel = rel == 3                                  # half an ulp of a (or just around it)
    ea = (a["se"][sel] & 0x7fff).astype(np.int64)
    eb = np.clip(ea - rng.integers(63, 66, sel.sum()), 0, 0x7ffe)
    b["m"][sel] = np.uint64(1 << 63) | (rng.integers(0, 2, sel.sum(), dtype=np.uint64) *
                                        rng.integers(0, 1 << 20, sel.sum(), dtype=np.uint64))
    b["se"][sel] = (eb | (rng.integers(0, 2, sel.sum()) << 15)).astype(np.uint16)
    return b, a


def xfi_operands(n, seed):
    """MPI_LONG_DOUBLE_INT (in, inout) pairs: x87 values with ties and small locs."""
    rng = np.random.default_rng(seed + 7)
    b, a = xf_operands(n, seed)
    outs = []
    for v in (b, a):
        o = np.zeros(n, XFI_DT)
        for f in ("m", "se", "pad0", "pad1"):
            o[f] = v[f]
        o["l"] = rng.integers(-3, 20, n)
        for f in ("pa", "pb", "pc"):
            o[f] = rng.integers(-(1 << 31), 1 << 31, n)
        outs.append(o)
    return outs[0], outs[1]
