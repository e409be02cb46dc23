"""CPU: libmvx.so's per-rank plans reproduce the reference's schedules.

Every rank's plan (mvx_plan_build) is executed on the CPU with the oracle op
(tests/plan_exec.py) and compared with oracle/coll_sim.c, which replays the
reference's intra_fns_new.c message schedule.  Bit-exact, NaN and signed
zeros included (both sides run the same x86 op code).
"""
import numpy as np
import pytest

from plan_exec import run_plans

import mvxtest as T

CASES = [(102, 10), (100, 10), (101, 10), (101, 11), (103, 11), (111, 17), (110, 17), (110, 18), (111, 19),
         (111, 20), (110, 21), (105, 8), (108, 4), (102, 6), (102, 23), (103, 24), (109, 3),
         (102, 12), (103, 12), (100, 12), (104, 12), (111, 22), (110, 22)]


def special_vec(dtype, n, seed):
    v = T.rand_vec(dtype, n, seed)
    rng = np.random.default_rng(seed + 1)
    if v.dtype.names and v.dtype.fields["v"][0].kind == "f":
        sp = np.array([np.nan, 0.0, -0.0, np.inf, 1.0], v.dtype.fields["v"][0])
        m = rng.random(n) < 0.2
        v["v"][m] = sp[rng.integers(0, sp.size, int(m.sum()))]
    elif v.dtype.kind == "f":
        sp = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf, 1.0], v.dtype)
        m = rng.random(n) < 0.2
        v[m] = sp[rng.integers(0, sp.size, int(m.sum()))]
    return v


def _cmp(op, dtype, got_u8, ref):
    T.assert_same(op, dtype, got_u8.view(np.uint8), ref, typemap_only=True)


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("op,dtype", CASES)
def test_allreduce_plans(mvx, oracle, p, op, dtype):
    for n in (1, 5, 10, 300, 2047, 2049, 16400, 70000):
        S = [special_vec(dtype, n, 1000 * p + 31 * r + n) for r in range(p)]
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        rc = oracle.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op)
        plans = [mvx.plan(mvx.COLL_ALLREDUCE, p, r, n, dtype, op) for r in range(p)]
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in range(p):
            _cmp(op, dtype, R1[r], R0[r])
        assert rc == [0] * p


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("op,dtype", CASES[::2])
def test_reduce_plans(mvx, oracle, p, op, dtype):
    for n in (1, 7, 1025, 4096, 40000):
        for root in sorted({0, 1 % p, p - 1, p // 2}):
            S = [special_vec(dtype, n, 77 * p + 13 * r + n + root) for r in range(p)]
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            oracle.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op, root)
            plans = [mvx.plan(mvx.COLL_REDUCE, p, r, n, dtype, op, root) for r in range(p)]
            R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
            _cmp(op, dtype, R1[root], R0[root])


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("op,dtype", CASES[1::2])
def test_reduce_scatter_plans(mvx, oracle, p, op, dtype):
    E = T.rand_vec(dtype, 1, 0).dtype.itemsize
    for base in (0, 1, 2, 100, 9000, 70000):
        cnts = [max(0, base + (r % 3) - 1) for r in range(p)]
        tot = sum(cnts)
        S = [special_vec(dtype, max(tot, 1), 5 * p + r + base) for r in range(p)]
        R0 = [np.zeros(max(c, 1), S[0].dtype) for c in cnts]
        oracle.reduce_scatter([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], cnts, dtype, op)
        plans = [mvx.plan(mvx.COLL_REDUCE_SCATTER, p, r, 0, dtype, op, 0, cnts) for r in range(p)]
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(max(c, 1) * E, np.uint8) for c in cnts])
        for r in range(p):
            if cnts[r]:
                _cmp(op, dtype, R1[r][: cnts[r] * E], R0[r][: cnts[r]])


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("op,dtype", CASES)
def test_scan_plans(mvx, oracle, p, op, dtype):
    """MPI_Scan: rank r's chain of balanced trees (intra_scan.c:118-147)."""
    for n in (1, 9, 3000):
        S = [special_vec(dtype, n, 3 * p + 11 * r + n) for r in range(p)]
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        rc = oracle.scan([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op)
        plans = [mvx.plan(mvx.COLL_SCAN, p, r, n, dtype, op) for r in range(p)]
        assert [P.k for P in plans] == [r + 1 for r in range(p)]
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in range(p):
            _cmp(op, dtype, R1[r], R0[r])
        assert rc == [0] * p


def test_scan_undefined_op_is_not_an_error(oracle):
    """MPIR_intra_Scan never reports MPIR_Op_errno (intra_scan.c:143-150)."""
    x = [np.arange(4, dtype=np.float32).view(np.uint8) for _ in range(4)]
    y = [np.zeros(4, np.float32).view(np.uint8) for _ in range(4)]
    assert oracle.scan(x, y, 4, 10, 105) == [0] * 4
    assert all(np.array_equal(a, b) for a, b in zip(x, y))


def test_algorithm_thresholds(mvx, oracle):
    """coll_table (intra_fns_new.c:129-132) and the Reduce_scatter 512 KiB
    switch (:39, :6248): plan and oracle agree at and around every edge."""
    A = mvx
    for coll in (A.COLL_ALLREDUCE, A.COLL_REDUCE, A.COLL_REDUCE_SCATTER):
        for p in range(1, 9):
            for dtype in (10, 11, 17, 18, 20, 1):
                for nbytes in (4, 4096, 8192, 16384, 65536, 65540, 524284, 524288, 1 << 20):
                    e, ts = mvx.dtype_info(dtype)
                    for n in {max(nbytes // ts - 1, 1), max(nbytes // ts, 1), nbytes // ts + 1, 3}:
                        assert mvx.algorithm(coll, p, n, dtype) == oracle.algorithm(coll, p, n, dtype)
    # facts from SURVEY.md section 2.3 / BASELINE configs
    assert mvx.algorithm(A.COLL_ALLREDUCE, 2, 1 << 26, 10) == A.ALG_RECDBL          # p = 2: always doubling
    assert mvx.algorithm(A.COLL_ALLREDUCE, 8, 1 << 26, 10) == A.ALG_RABENSEIFNER    # C3
    assert mvx.algorithm(A.COLL_ALLREDUCE, 8, 2047, 10) == A.ALG_RECDBL             # < 8 KiB at p = 8
    assert mvx.algorithm(A.COLL_ALLREDUCE, 8, 2048, 10) == A.ALG_RABENSEIFNER
    assert mvx.algorithm(A.COLL_ALLREDUCE, 4, 16383, 10) == A.ALG_RECDBL            # < 64 KiB at p = 4
    assert mvx.algorithm(A.COLL_REDUCE, 8, 1024, 10) == A.ALG_BINOMIAL              # strict > 4096 at p = 8
    assert mvx.algorithm(A.COLL_REDUCE, 8, 1025, 10) == A.ALG_RABENSEIFNER
    assert mvx.algorithm(A.COLL_REDUCE, 4, 16385, 10) == A.ALG_RABENSEIFNER         # > 64 KiB at p = 4
    assert mvx.algorithm(A.COLL_REDUCE, 2, 1 << 20, 6) == A.ALG_BINOMIAL            # C1
    assert mvx.algorithm(A.COLL_REDUCE_SCATTER, 4, 1 << 27, 8) == A.ALG_RS_PAIRWISE  # C4: 1 GiB total
    assert mvx.algorithm(A.COLL_REDUCE_SCATTER, 4, 1 << 28, 8) == A.ALG_RS_HALVING   # 2 GiB: int32 wrap
    assert mvx.algorithm(A.COLL_ALLREDUCE, 8, 1 << 26, 17) == A.ALG_RABENSEIFNER    # C5


@pytest.mark.parametrize("p", range(1, 9))
def test_calls_uop_matches_reference_error_codes(mvx, oracle, p):
    """An undefined (op, type) pair is reported exactly by the ranks on which
    the reference calls (*uop) (A.5: p = 1 returns 0)."""
    for coll, n in ((mvx.COLL_ALLREDUCE, 5), (mvx.COLL_ALLREDUCE, 5000), (mvx.COLL_REDUCE, 5),
                    (mvx.COLL_REDUCE, 5000), (mvx.COLL_REDUCE_SCATTER, 3), (mvx.COLL_REDUCE_SCATTER, 70000)):
        roots = range(p) if coll == mvx.COLL_REDUCE else [0]
        for root in roots:
            cnts = [n + (r % 2) for r in range(p)] if coll == mvx.COLL_REDUCE_SCATTER else None
            tot = sum(cnts) if cnts else n
            S = [np.zeros(tot, np.float32).view(np.uint8) for _ in range(p)]
            R = [np.zeros(tot, np.float32).view(np.uint8) for _ in range(p)]
            if coll == mvx.COLL_ALLREDUCE:
                rc = oracle.allreduce(S, R, n, 10, 105)
            elif coll == mvx.COLL_REDUCE:
                rc = oracle.reduce(S, R, n, 10, 105, root)
            else:
                rc = oracle.reduce_scatter(S, R, cnts, 10, 105)
            calls = [mvx.plan(coll, p, r, n, 10, 105, root, cnts).calls_uop for r in range(p)]
            assert rc == [329 if c else 0 for c in calls], (coll, n, root, rc, calls)
