"""CPU: libmvx.so's plans for user-defined ops reproduce the reference.

For MPI_Op_create ops the reference changes algorithm (permanent == 0:
recursive doubling / binomial, intra_fns_new.c:5590, 4620) and, for a
noncommutative op, operand roles (5610-5624, 4908-4966, 6487-6498,
6505-6706, intra_scan.c:124-137).  Each rank's plan (mvx_plan_build_kind)
runs on the CPU with the same C user function (tests/user_ops.c) that the
oracle's replay calls; results must be bit-identical.  `mix` is neither
commutative nor associative, so any difference in grouping or operand role
shows; it is tested under both commute flags (a user may declare a
noncommutative function commutative; the reference then just takes the
commutative branches).
"""
import numpy as np
import pytest

import uops
from plan_exec import run_plans

H = 240
KINDS = {1: 1, 0: 2}   # commute flag -> OPKIND


def _sends(name, p, n, seed):
    return [uops.rand_for(name, n, seed + 7 * r) for r in range(p)]


def _setup(oracle, name, commute):
    assert oracle.user_op_set(H, uops.host_fn(name), commute) == 0
    return uops.UOPS[name][0], KINDS[commute]


CASES = [("mix", 0), ("mix", 1), ("affine", 0), ("fsum", 1), ("fsum", 0), ("addem", 1)]


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("name,commute", CASES)
def test_user_allreduce_plans(mvx, oracle, p, name, commute):
    dt, kind = _setup(oracle, name, commute)
    for n in (1, 3, 64, 1000, 5001):
        S = _sends(name, p, n, 100 * p + n)
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        assert oracle.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dt, H) == [0] * p
        plans = [mvx.plan(mvx.COLL_ALLREDUCE, p, r, n, dt, H, opkind=kind) for r in range(p)]
        assert plans[0].alg == mvx.ALG_RECDBL
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in range(p):
            assert np.array_equal(R1[r].view(S[0].dtype), R0[r]), (n, r)


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("name,commute", CASES)
def test_user_reduce_plans(mvx, oracle, p, name, commute):
    dt, kind = _setup(oracle, name, commute)
    for n in (1, 17, 3000):
        for root in sorted({0, p - 1, p // 2}):
            S = _sends(name, p, n, 50 * p + n + root)
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            oracle.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dt, H, root)
            plans = [mvx.plan(mvx.COLL_REDUCE, p, r, n, dt, H, root, opkind=kind) for r in range(p)]
            assert plans[0].alg == mvx.ALG_BINOMIAL
            R1 = run_plans(plans, [s.view(np.uint8) for s in S],
                           [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
            assert np.array_equal(R1[root].view(S[0].dtype), R0[root]), (n, root)


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("name,commute", CASES)
def test_user_scan_plans(mvx, oracle, p, name, commute):
    dt, kind = _setup(oracle, name, commute)
    for n in (1, 100, 2001):
        S = _sends(name, p, n, 30 * p + n)
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        oracle.scan([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dt, H)
        plans = [mvx.plan(mvx.COLL_SCAN, p, r, n, dt, H, opkind=kind) for r in range(p)]
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in range(p):
            assert np.array_equal(R1[r].view(S[0].dtype), R0[r]), (n, r)


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("name,commute", CASES)
def test_user_reduce_scatter_plans(mvx, oracle, p, name, commute):
    dt, kind = _setup(oracle, name, commute)
    E = np.dtype(uops.UOPS[name][2]).itemsize
    seen = set()
    for base in (0, 1, 2, 5, 30, 200, 20000):
        cnts = [max(0, base + (r % 3) - 1) for r in range(p)]
        total = sum(cnts)
        if total == 0:
            continue
        S = _sends(name, p, total, 9 * p + base)
        R0 = [np.zeros(max(c, 1), S[0].dtype) for c in cnts]
        oracle.reduce_scatter([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], cnts, dt, H)
        plans = [mvx.plan(mvx.COLL_REDUCE_SCATTER, p, r, 0, dt, H, recvcnts=cnts, opkind=kind) for r in range(p)]
        assert plans[0].alg == oracle.algorithm(3, p, total, dt, H)
        seen.add(plans[0].alg)
        R1 = run_plans(plans, [s.view(np.uint8) for s in S],
                       [np.zeros(max(c, 1) * E, np.uint8) for c in cnts])
        for r in range(p):
            assert np.array_equal(R1[r][: cnts[r] * E].view(S[0].dtype), R0[r][: cnts[r]]), (base, r, cnts)
    if p > 1 and commute == 0:
        assert seen == {mvx.ALG_RS_RECDBL, mvx.ALG_RS_PAIRWISE}
