"""Test helpers for derived contiguous datatypes (MPI_Type_contiguous).

The product's type table (libmvx_hip.so) and the oracle's (oracle/cpu_ops.c)
are separate; `make_both` creates a type in both and checks they agree on
the handle, extent and size, so one handle names the same type on each side.
"""
import numpy as np

import mvxtest as T

# base handle -> numpy scalar type of a {value, loc} stride-2 pair
PAIR_BASES = {1: np.int8, 4: np.int16, 6: np.int32, 8: np.int64, 13: np.int64, 10: np.float32,
              11: np.float64, 12: np.longdouble,
              28: np.int32, 26: np.float32, 27: np.float64}    # MPI_INTEGER / REAL / DOUBLE_PRECISION


def make_both(mvx, oracle, count, old):
    rc, h = mvx.MPI_Type_contiguous(count, old)
    orc, oh = oracle.type_contiguous(count, old)
    assert (rc, h) == (orc, oh), (count, old, rc, h, orc, oh)
    if rc == 0:
        assert mvx.MPI_Type_extent(h)[1] == oracle.dtype_info(h)[0]
        assert mvx.MPI_Type_size(h)[1] == oracle.dtype_info(h)[1]
    return rc, h


def free_both(mvx, oracle, h):
    assert mvx.MPI_Type_free(h)[0] == 0
    assert oracle.type_free(h) == 0


def pair_dtype(base):
    t = np.dtype(PAIR_BASES[base])
    return np.dtype([("v", t), ("l", t)])


def rand_pairs(base, n, seed):
    """{value, loc} pairs of one base type with many value ties (and NaN /
    +-0 / inf for the float bases, every x87 class for long double)."""
    rng = np.random.default_rng(seed)
    if base == 12:
        out = np.zeros(n, pair_dtype(12))
        u = out.view(np.uint8).reshape(n, 32)
        u[:, :16] = T.xf_rand(n, rng).view(np.uint8).reshape(n, 16)
        u[:, 16:] = T.xf_rand(n, rng).view(np.uint8).reshape(n, 16)
        ties = rng.random(n) < 0.3                      # equal values: loc tie-break
        u[ties, :16] = u[np.roll(np.arange(n), 1)[ties], :16]
        return out
    dt = pair_dtype(base)
    out = np.zeros(n, dt)
    t = dt.fields["v"][0]
    if t.kind == "f":
        v = rng.integers(-4, 5, n).astype(t)
        l = (rng.standard_normal(n) * 100).astype(t)
        sp = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf], t)
        for arr in (v, l):
            m = rng.random(n) < 0.1
            arr[m] = sp[rng.integers(0, sp.size, int(m.sum()))]
        out["v"], out["l"] = v, l
    else:
        info = np.iinfo(t)
        out["v"] = rng.integers(-4, 5, n).astype(t)
        out["l"] = rng.integers(info.min, info.max, n, dtype=t, endpoint=True)
    return out


def assert_pairs_same(got_u8, ref):
    """Bit-exact on the type map (value and loc; the long-double slots whole,
    padding included, as the op writes 10 bytes and keeps inout's 6)."""
    got = np.asarray(got_u8).view(np.uint8)[: ref.nbytes]
    assert np.array_equal(got, np.ascontiguousarray(ref).view(np.uint8)), "pairs differ"
