"""CPU: derived contiguous datatypes (MPI_Type_contiguous and friends).

Reference: src/pt2pt/type_contig.c:52-187 (checks 66-75, flattening
139-146, extent/size 149-169), type_free.c:60-105, and the ops' treatment of
a derived type -- MAXLOC / MINLOC on a count-2 contiguous type over INT,
LONG, LONG_LONG_INT, SHORT, CHAR, FLOAT, DOUBLE or LONG_DOUBLE take stride-2
{value, loc} pairs (global_ops.c:1387-1503, 1625-1740); every other op has no
MPIR_CONTIG case and answers 329.

Pinning: the oracle restates those lines (oracle/cpu_ops.c); a count-2
contiguous type over MPI_INT must reduce exactly like the reference's own
MPI_2INT (which initdte.c:167 builds with the same call) -- checked against
the oracle's MPI_2INT path, which allred.c-style cases pin; the plans with a
derived type are checked against the oracle's replay of the schedules.
"""
import numpy as np
import pytest

import derived_util as D
import uops
from plan_exec import run_plans

# the Fortran types too: INTEGER / REAL / DOUBLE_PRECISION (pair bases by
# their dte_type), LOGICAL, and the predefined pairs 2INTEGER / 2REAL
BASES = [1, 2, 3, 4, 6, 7, 8, 13, 10, 11, 12, 17, 18, 21, 23, 25, 26, 27, 28, 29, 32]


def test_contiguous_facts_match_the_reference(mvx, oracle):
    """Extent, size, flattening and error codes of type_contig.c, both
    tables side by side."""
    made = []
    for old in BASES:
        for count in (0, 1, 2, 3):
            rc, h = D.make_both(mvx, oracle, count, old)
            assert rc == 0
            made.append(h)
            e, s = mvx.dtype_info(old)
            assert mvx.MPI_Type_extent(h) == (0, count * e)
            assert mvx.MPI_Type_size(h) == (0, count * s)
    # flattening: contig(1, MPI_2INT) = contig(2, INT) -> a MAXLOC pair type;
    # the Fortran pairs flatten to the old type initfutil.c built them over
    for pair, flat in ((21, 6), (29, 28), (32, 10), (33, 11), (30, 23)):
        rc, h = D.make_both(mvx, oracle, 1, pair)
        made.append(h)
        assert _describe(mvx, h) == (flat, 2)
    rc, h2 = D.make_both(mvx, oracle, 2, made[0 * 4 + 1])    # contig(2, contig(1, CHAR))
    made.append(h2)
    assert _describe(mvx, h2) == (1, 2)
    # a type over a padded struct is not contiguous: no flattening below it
    rc, h3 = D.make_both(mvx, oracle, 3, 18)                  # contig(3, DOUBLE_INT)
    rc, h4 = D.make_both(mvx, oracle, 1, h3)
    made += [h3, h4]
    assert _describe(mvx, h4) == (h3, 1)
    assert mvx.MPI_Type_extent(h4) == (0, 48) and mvx.MPI_Type_size(h4) == (0, 36)
    # errors: count < 0, MPI_UB / MPI_LB, null or unknown old type
    assert mvx.MPI_Type_contiguous(-1, 10)[0] == oracle.type_contiguous(-1, 10)[0] == 2
    assert mvx.MPI_Type_contiguous(2, 16)[0] == oracle.type_contiguous(2, 16)[0] == 3
    assert mvx.MPI_Type_contiguous(2, 15)[0] == 3
    assert mvx.MPI_Type_contiguous(2, 0)[0] == oracle.type_contiguous(2, 0)[0] == 323
    assert mvx.MPI_Type_contiguous(2, 99)[0] == 323
    assert mvx.MPI_Type_commit(made[0]) == 0 and mvx.MPI_Type_commit(99) == 323
    # free: predefined 579, null 323, derived -> MPI_DATATYPE_NULL
    assert mvx.MPI_Type_free(10) == (579, 10)
    assert mvx.MPI_Type_free(0)[0] == 323
    for h in made:
        D.free_both(mvx, oracle, h)
    assert mvx.MPI_Type_extent(made[0])[0] == 323


def _describe(mvx, h):
    import ctypes
    o, c = ctypes.c_int(), ctypes.c_int()
    assert mvx.hip().mvx_type_describe(h, ctypes.byref(o), ctypes.byref(c), None, None) == 0
    return o.value, c.value


def test_op_support_on_derived_types(mvx, oracle):
    """Every predefined op on a spread of derived types: the device verdict
    is the oracle's (MAXLOC / MINLOC on count-2 pairs of the eight bases, 329
    everywhere else)."""
    made = []
    try:
        for old in BASES + [5, 9, 24, 20]:
            for count in (1, 2, 4):
                rc, h = D.make_both(mvx, oracle, count, old)
                made.append(h)
                for op in range(100, 112):
                    ref = oracle.op(op, h, np.zeros(256, np.uint8), np.zeros(256, np.uint8), 1)
                    got = mvx.hip().mvx_op_apply(op, h, None, None, 0, None)
                    assert got == ref, (old, count, op, got, ref)
                    fo, fc = _describe(mvx, h)     # after flattening (contig(1, 2INT) = 2 x INT)
                    ok = op in (110, 111) and fc == 2 and fo in D.PAIR_BASES
                    assert (ref == 0) == ok, (old, count, op)
    finally:
        for h in made:
            D.free_both(mvx, oracle, h)


def test_int_pair_is_mpi_2int(mvx, oracle):
    """contig(2, MPI_INT) reduces exactly as MPI_2INT (initdte.c:167 builds
    MPI_2INT with that call)."""
    rc, h = D.make_both(mvx, oracle, 2, 6)
    try:
        a, b = D.rand_pairs(6, 5000, 1), D.rand_pairs(6, 5000, 2)
        for op in (110, 111):
            r1, r2 = b.copy(), b.copy()
            assert oracle.op(op, h, a.view(np.uint8), r1.view(np.uint8), a.size) == 0
            assert oracle.op(op, 21, a.view(np.uint8), r2.view(np.uint8), a.size) == 0
            assert np.array_equal(r1.view(np.uint8), r2.view(np.uint8))
    finally:
        D.free_both(mvx, oracle, h)


@pytest.mark.parametrize("base", sorted(D.PAIR_BASES))
def test_pair_semantics_restated(oracle, mvx, base):
    """The oracle's stride-2 loop on a few hand-made cases: equal values ->
    the smaller loc (MPIR_MIN, NaN-in-accumulator kept); strictly larger
    (smaller) value -> both of b's; NaN values never replace."""
    if base == 12:
        pytest.skip("x87 pairs are covered by the device fuzz against the oracle")
    rc, h = D.make_both(mvx, oracle, 2, base)
    try:
        dt = D.pair_dtype(base)
        t = dt.fields["v"][0].type
        a = np.zeros(4, dt)
        b = np.zeros(4, dt)
        a["v"], a["l"] = [t(1), t(2), t(3), t(3)], [t(5), t(5), t(5), t(1)]
        b["v"], b["l"] = [t(1), t(3), t(2), t(3)], [t(2), t(9), t(9), t(4)]
        r = a.copy()
        assert oracle.op(111, h, b.view(np.uint8), r.view(np.uint8), 4) == 0
        assert list(r["v"]) == [1, 3, 3, 3] and list(r["l"]) == [2, 9, 5, 1]
        r = a.copy()
        assert oracle.op(110, h, b.view(np.uint8), r.view(np.uint8), 4) == 0
        assert list(r["v"]) == [1, 2, 2, 3] and list(r["l"]) == [2, 5, 9, 1]
    finally:
        D.free_both(mvx, oracle, h)


COLLS = [(1, 111, 10), (1, 110, 11), (1, 111, 6), (2, 110, 1), (2, 111, 8), (3, 111, 4), (3, 110, 10),
         (1, 111, 13), (2, 110, 12), (1, 110, 26), (3, 111, 27), (2, 111, 28)]


@pytest.mark.parametrize("p", [1, 2, 3, 4, 6, 8])
@pytest.mark.parametrize("coll,op,base", COLLS)
def test_plans_with_derived_pairs(mvx, oracle, p, coll, op, base):
    """Collectives on a derived MAXLOC / MINLOC type: every rank's plan
    against the oracle's replay (roles matter for the float bases)."""
    rc, h = D.make_both(mvx, oracle, 2, base)
    try:
        E = D.pair_dtype(base).itemsize
        for n in (1, 9, 1000, 40000):
            S = [D.rand_pairs(base, n, 31 * p + 7 * r + n) for r in range(p)]
            sb = [s.view(np.uint8) for s in S]
            if coll == 3:
                cnts = [n // p + (r % 2) for r in range(p)]
                tot = sum(cnts)
                S = [D.rand_pairs(base, tot, 5 * p + r + n) for r in range(p)]
                sb = [s.view(np.uint8) for s in S]
                R0 = [np.zeros(max(c, 1), S[0].dtype) for c in cnts]
                oracle.reduce_scatter(sb, [x.view(np.uint8) for x in R0], cnts, h, op)
                plans = [mvx.plan(coll, p, r, 0, h, op, 0, cnts) for r in range(p)]
                R1 = run_plans(plans, sb, [np.zeros(max(c, 1) * E, np.uint8) for c in cnts])
                for r in range(p):
                    D.assert_pairs_same(R1[r][: cnts[r] * E], R0[r][: cnts[r]])
                continue
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            root = p - 1
            if coll == 1:
                rcs = oracle.allreduce(sb, [x.view(np.uint8) for x in R0], n, h, op)
            else:
                rcs = oracle.reduce(sb, [x.view(np.uint8) for x in R0], n, h, op, root)
            assert rcs == [0] * p
            plans = [mvx.plan(coll, p, r, n, h, op, root) for r in range(p)]
            R1 = run_plans(plans, sb, [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
            for r in (range(p) if coll == 1 else [root]):
                D.assert_pairs_same(R1[r], R0[r])
    finally:
        D.free_both(mvx, oracle, h)


def test_undefined_op_on_derived_type_is_329(mvx, oracle):
    """SUM on contig(4, MPI_FLOAT): 329 on the ranks that call (*uop)."""
    rc, h = D.make_both(mvx, oracle, 4, 10)
    try:
        p, n = 4, 100
        x = [np.zeros(16 * n, np.uint8) for _ in range(p)]
        y = [np.zeros(16 * n, np.uint8) for _ in range(p)]
        rcs = oracle.allreduce(x, y, n, h, 102)
        calls = [mvx.plan(1, p, r, n, h, 102).calls_uop for r in range(p)]
        assert rcs == [329 if c else 0 for c in calls] == [329] * p
    finally:
        D.free_both(mvx, oracle, h)


@pytest.mark.parametrize("p", [2, 3, 5, 8])
def test_user_op_with_derived_type(mvx, oracle, p):
    """A user function over a derived type gets the derived handle and the
    count of derived elements (the reference's (*uop)(.., &len, &type));
    the schedules move count * extent bytes.  (A function must be element-
    wise over its datatype's elements, MPI-1.2 section 4.9.4: the plans may
    hand it any block of whole elements.)"""
    rc, h = D.make_both(mvx, oracle, 3, 7)          # 3 x MPI_UNSIGNED, 12 bytes
    H = 240
    try:
        assert oracle.user_op_set(H, uops.host_fn("mix3"), 0) == 0
        for n in (1, 7, 500):
            S = [np.random.default_rng(9 * p + r + n).integers(0, 1 << 32, 3 * n, dtype=np.uint64).astype(np.uint32)
                 for r in range(p)]
            sb = [s.view(np.uint8) for s in S]
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            oracle.allreduce(sb, [x.view(np.uint8) for x in R0], n, h, H)
            plans = [mvx.plan(1, p, r, n, h, H, opkind=2) for r in range(p)]
            assert plans[0].esize == 12
            R1 = _run_user_plans(plans, sb, n, h, H)
            for r in range(p):
                assert np.array_equal(R1[r], R0[r].view(np.uint8)), (n, r)
    finally:
        D.free_both(mvx, oracle, h)


def _run_user_plans(plans, sb, n, h, H):
    """run_plans with the oracle's user op: leaves are n derived elements,
    the function sees the derived handle."""
    return run_plans(plans, sb, [np.zeros(sb[0].size, np.uint8) for _ in plans])
