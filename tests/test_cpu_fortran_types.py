"""CPU: the Fortran datatypes of a Fortran-enabled build (mpi.h:101-113).

MPI_Init registers them for C callers too (initutil.c:421-422 ->
MPIR_InitFortranDatatypes, src/fortran/src/initfutil.c:220-349):

* MPI_INTEGER / MPI_REAL / MPI_DOUBLE_PRECISION are base types whose
  dte_type is MPIR_INT / MPIR_FLOAT / MPIR_DOUBLE, so every op treats them as
  int / float / double.
* MPI_LOGICAL (dte_type MPIR_LOGICAL, one MPI_Fint) has the logical ops
  through FROM_FLOG / TO_FLOG (global_ops.c:646-655, 875-884, 1104-1113;
  mpi_fort.h:11-19) and the bitwise ops on the word (678-684, 906-912,
  1136-1142).  Everything else is 329.
* MPI_2INTEGER / 2REAL / 2DOUBLE_PRECISION / 2COMPLEX / 2DOUBLE_COMPLEX are
  contiguous(2, x).  MAXLOC / MINLOC run the stride-2 case of x's dte_type
  (1387-1503); there is no case for COMPLEX.

Pinning: allredf.f's known answers (tests/golden/known_answers.json, "other",
checked against the oracle by test_cpu_oracle.py) and the restatements below.
"""
import numpy as np
import pytest

import derived_util as D
import mvxtest as T
from plan_exec import run_plans

LOGICAL, REAL, DPREC, INTEGER = 25, 26, 27, 28
P2INTEGER, P2COMPLEX, P2DCOMPLEX, P2REAL, P2DPREC = 29, 30, 31, 32, 33


def _apply(oracle, op, dtype, a, b):
    r = T.clone(b)
    rc = oracle.op(op, dtype, a.view(np.uint8), r.view(np.uint8), a.size)
    return rc, r


@pytest.mark.parametrize("flog", [(1, 0), (-1, 0), (7, 3)])
def test_logical_ops_restated(oracle, flog):
    """LAND / LOR / LXOR compare each word with .TRUE. only (any other word,
    .FALSE. or not, is false) and store .TRUE. / .FALSE.; BAND / BOR / BXOR
    act on the bits; the other ops are 329."""
    t, f = flog
    oracle.set_fortran_logical(t, f)
    try:
        rng = np.random.default_rng(5)
        words = np.array([t, f, 0, 1, -1, 2, t, f], np.int32)
        a = rng.choice(words, 4000)
        b = rng.choice(words, 4000)
        ta, tb = a == t, b == t
        want = {104: ta & tb, 106: ta | tb, 108: ta ^ tb}
        for op, v in want.items():
            rc, r = _apply(oracle, op, LOGICAL, b, a)      # inout = a
            assert rc == 0
            assert np.array_equal(r, np.where(v, t, f).astype(np.int32)), op
        for op, fn in ((105, np.bitwise_and), (107, np.bitwise_or), (109, np.bitwise_xor)):
            rc, r = _apply(oracle, op, LOGICAL, b, a)
            assert rc == 0 and np.array_equal(r, fn(a, b)), op
        for op in (100, 101, 102, 103, 110, 111):
            assert _apply(oracle, op, LOGICAL, b, a)[0] == 329
    finally:
        oracle.set_fortran_logical(1, 0)


@pytest.mark.parametrize("fort,c", [(INTEGER, 6), (REAL, 10), (DPREC, 11), (P2INTEGER, 21)])
def test_fortran_types_reduce_as_their_c_twins(oracle, fort, c):
    """Same dte_type, same bits: INTEGER = INT, REAL = FLOAT, DOUBLE_PRECISION
    = DOUBLE, 2INTEGER = 2INT (contiguous(2, INTEGER) over MPIR_INT), for
    every op, including the 329 verdicts."""
    a, b = T.rand_vec(c, 3000, 1), T.rand_vec(c, 3000, 2)
    for op in range(100, 112):
        r1 = _apply(oracle, op, fort, a, b)
        r2 = _apply(oracle, op, c, a, b)
        assert r1[0] == r2[0], op
        assert np.array_equal(r1[1].view(np.uint8), r2[1].view(np.uint8)), op


@pytest.mark.parametrize("pair,base", [(P2REAL, 10), (P2DPREC, 11)])
def test_float_pairs_are_contiguous_pairs(mvx, oracle, pair, base):
    """2REAL / 2DOUBLE_PRECISION reduce as a user's contiguous(2, FLOAT /
    DOUBLE): the same loop (global_ops.c:1459-1482), float locs included."""
    rc, h = D.make_both(mvx, oracle, 2, base)
    try:
        a, b = D.rand_pairs(base, 5000, 3), D.rand_pairs(base, 5000, 4)
        for op in (110, 111):
            r1, r2 = _apply(oracle, op, pair, a, b), _apply(oracle, op, h, a, b)
            assert r1[0] == r2[0] == 0
            assert np.array_equal(r1[1].view(np.uint8), r2[1].view(np.uint8))
        for op in (100, 102, 105):
            assert _apply(oracle, op, pair, a, b)[0] == 329
    finally:
        D.free_both(mvx, oracle, h)


def test_complex_pairs_have_no_case(mvx, oracle):
    """contiguous(2, COMPLEX / DOUBLE_COMPLEX): no dte_type case in MAXLOC /
    MINLOC (1498-1501), none in any other op: 329 on the device verdict and
    the oracle alike."""
    for t in (P2COMPLEX, P2DCOMPLEX):
        for op in range(100, 112):
            assert T.oracle_rc(oracle, op, t) == 329
            assert mvx.hip().mvx_op_apply(op, t, None, None, 0, None) == 329


def test_struct_over_fortran_first_member(mvx, oracle):
    """MAXLOC on an MPIR_STRUCT reads the C pair struct of old_types[0]'s
    dte_type (1280-1384): {INTEGER, INTEGER} is MPIR_2int_loctype, {REAL,
    INTEGER} MPIR_floatint_loctype, {LOGICAL, INTEGER} has no case."""
    made = []
    try:
        for first, want in ((INTEGER, 0), (REAL, 0), (LOGICAL, 329)):
            rm, hm = mvx.MPI_Type_struct(2, [1, 1], [0, 4], [first, 6])
            ro, ho = oracle.type_struct(2, [1, 1], [0, 4], [first, 6])
            assert rm == ro == 0 and hm == ho
            made.append(hm)
            assert mvx.MPI_Type_commit(hm) == 0 and oracle.type_commit(ho) == 0
            for op in (110, 111):
                assert T.oracle_rc(oracle, op, hm) == want
                assert mvx.hip().mvx_op_apply(op, hm, None, None, 0, None) == want
            if want == 0:
                c = 21 if first == INTEGER else 17
                a, b = T.rand_vec(c, 2000, 8), T.rand_vec(c, 2000, 9)
                for op in (110, 111):
                    r1, r2 = _apply(oracle, op, hm, a, b), _apply(oracle, op, c, a, b)
                    assert np.array_equal(r1[1].view(np.uint8), r2[1].view(np.uint8))
    finally:
        for h in made:
            assert mvx.MPI_Type_free(h)[0] == 0 and oracle.type_free(h) == 0


CASES = [(1, 100, REAL), (2, 101, DPREC), (3, 102, REAL), (1, 108, LOGICAL), (2, 104, LOGICAL),
         (1, 111, P2REAL), (2, 110, P2DPREC), (3, 111, P2INTEGER), (1, 109, INTEGER)]


@pytest.mark.parametrize("p", [2, 3, 5, 8])
@pytest.mark.parametrize("coll,op,dtype", CASES)
def test_plans_with_fortran_types(mvx, oracle, p, coll, op, dtype):
    """Every rank's plan against the oracle's replay of the reference's
    schedules.  The float types keep their operand roles (NaN, +-0), as
    MPI_FLOAT does: REAL's MAX and 2REAL's MAXLOC are not symmetric."""
    E = mvx.NP_DTYPE[dtype].itemsize
    for n in (1, 9, 1000, 40000):
        S = [T.rand_vec(dtype, n, 31 * p + 7 * r + n) for r in range(p)]
        if dtype in (P2REAL, P2DPREC):
            S = [D.rand_pairs(10 if dtype == P2REAL else 11, n, 13 * p + r + n).view(S[0].dtype) for r in range(p)]
        sb = [s.view(np.uint8) for s in S]
        if coll == 3:
            cnts = [n // p + (r % 2) for r in range(p)]
            tot = sum(cnts)
            S = [T.rand_vec(dtype, tot, 5 * p + r + n) for r in range(p)]
            sb = [s.view(np.uint8) for s in S]
            R0 = [np.zeros(max(c, 1), S[0].dtype) for c in cnts]
            rcs = oracle.reduce_scatter(sb, [x.view(np.uint8) for x in R0], cnts, dtype, op)
            assert rcs == [0] * p
            plans = [mvx.plan(coll, p, r, 0, dtype, op, 0, cnts) for r in range(p)]
            R1 = run_plans(plans, sb, [np.zeros(max(c, 1) * E, np.uint8) for c in cnts])
            for r in range(p):
                T.assert_same(op, dtype, R1[r][: cnts[r] * E], R0[r][: cnts[r]])
            continue
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        root = p - 1
        if coll == 1:
            rcs = oracle.allreduce(sb, [x.view(np.uint8) for x in R0], n, dtype, op)
        else:
            rcs = oracle.reduce(sb, [x.view(np.uint8) for x in R0], n, dtype, op, root)
        assert rcs == [0] * p
        plans = [mvx.plan(coll, p, r, n, dtype, op, root) for r in range(p)]
        R1 = run_plans(plans, sb, [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in (range(p) if coll == 1 else [root]):
            T.assert_same(op, dtype, R1[r], R0[r])


def test_symmetry_flags(mvx):
    """The plan may swap operands only where the result cannot tell: the
    float Fortran types pick by role under MAX / MIN / MAXLOC / MINLOC."""
    for dtype, op, sym in ((REAL, 100, 0), (DPREC, 101, 0), (INTEGER, 100, 1), (LOGICAL, 104, 1),
                           (P2REAL, 111, 0), (P2DPREC, 110, 0), (P2INTEGER, 111, 1), (REAL, 102, 1)):
        assert mvx.plan(1, 4, 0, 100, dtype, op).symmetric == sym, (dtype, op)
