"""CPU: communicators of more than 8 ranks (k > 8 combine leaves).

A launch combines at most 8 leaves (MVX_COMBINE_KMAX); the plan's program is
a chain of trees over up to 64 leaves, which the executor evaluates in groups
of 8.  Here every rank's plan runs on the CPU (tests/plan_exec.py) against
the oracle's replay of the reference schedule (oracle/coll_sim.c) for
p = 9 .. 64: the binomial Reduce (intra_fns_new.c:4907-4954), pairwise
Reduce_scatter (:6473-6500), Rabenseifner at pof2 = 16/32/64 and MPI_Scan on
ranks >= 8 (intra_scan.c:118-147).  The grouped evaluation itself is
checked against the one-pass program by tests/test_gpu_coll.py.
"""
import numpy as np
import pytest

from plan_exec import chain_mask, run_plans, tree_mask

import mvxtest as T

CASES = [(102, 10), (100, 10), (111, 17), (105, 8), (103, 11)]
PS = [9, 12, 16, 17, 31, 32, 33, 64]


def _cmp(op, dtype, got_u8, ref):
    T.assert_same(op, dtype, got_u8.view(np.uint8), ref, typemap_only=True)


@pytest.mark.parametrize("p", PS)
@pytest.mark.parametrize("op,dtype", CASES)
def test_allreduce_plans_wide(mvx, oracle, p, op, dtype):
    for n in (3, 200, 5000):
        S = [T.rand_vec(dtype, n, 1000 * p + 31 * r + n) for r in range(p)]
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        rc = oracle.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op)
        plans = [mvx.plan(mvx.COLL_ALLREDUCE, p, r, n, dtype, op) for r in range(p)]
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in range(p):
            _cmp(op, dtype, R1[r], R0[r])
        assert rc == [0] * p


@pytest.mark.parametrize("p", PS)
@pytest.mark.parametrize("op,dtype", CASES)
def test_reduce_plans_wide(mvx, oracle, p, op, dtype):
    for n in (5, 3000):
        for root in sorted({0, p - 1, p // 2}):
            S = [T.rand_vec(dtype, n, 77 * p + 13 * r + n + root) for r in range(p)]
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            oracle.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op, root)
            plans = [mvx.plan(mvx.COLL_REDUCE, p, r, n, dtype, op, root) for r in range(p)]
            R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
            _cmp(op, dtype, R1[root], R0[root])


@pytest.mark.parametrize("p", PS)
@pytest.mark.parametrize("op,dtype", CASES)
def test_reduce_scatter_plans_wide(mvx, oracle, p, op, dtype):
    E = T.rand_vec(dtype, 1, 0).dtype.itemsize
    for base in (1, 40, 9000):      # halving below 512 KiB total, pairwise above
        cnts = [max(0, base + (r % 3) - 1) for r in range(p)]
        tot = sum(cnts)
        S = [T.rand_vec(dtype, max(tot, 1), 5 * p + r + base) for r in range(p)]
        R0 = [np.zeros(max(c, 1), S[0].dtype) for c in cnts]
        oracle.reduce_scatter([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], cnts, dtype, op)
        plans = [mvx.plan(mvx.COLL_REDUCE_SCATTER, p, r, 0, dtype, op, 0, cnts) for r in range(p)]
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(max(c, 1) * E, np.uint8) for c in cnts])
        for r in range(p):
            if cnts[r]:
                _cmp(op, dtype, R1[r][: cnts[r] * E], R0[r][: cnts[r]])


@pytest.mark.parametrize("p", [9, 16, 33, 64])
@pytest.mark.parametrize("op,dtype", CASES[:3])
def test_scan_plans_wide(mvx, oracle, p, op, dtype):
    n = 257
    S = [T.rand_vec(dtype, n, 3 * p + 11 * r) for r in range(p)]
    R0 = [np.zeros_like(S[0]) for _ in range(p)]
    oracle.scan([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op)
    plans = [mvx.plan(mvx.COLL_SCAN, p, r, n, dtype, op) for r in range(p)]
    assert [P.k for P in plans] == [r + 1 for r in range(p)]
    R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
    for r in range(p):
        _cmp(op, dtype, R1[r], R0[r])


def test_single_launch_masks(mvx):
    """Up to 8 leaves the program is one launch: a TREE plan's masks are
    mvx_tree_mask(k), a CHAIN plan's mvx_chain_mask(k), and MPI_Scan's mix a
    tree per block plus a chain bit per block head."""
    for p in range(1, 9):
        P = mvx.plan(mvx.COLL_ALLREDUCE, p, 0, 1 << 20, 10, 102)
        assert P.masks() == (tree_mask(P.k), 0)
        P = mvx.plan(mvx.COLL_REDUCE_SCATTER, p, 0, 0, 10, 102, 0, [1 << 18] * p)
        assert P.masks() == (0, chain_mask(p))
    P = mvx.plan(mvx.COLL_SCAN, 8, 7, 10, 10, 102)      # [x7 | x6 | x5 x4 | x3 x2 x1 x0]
    assert P.segments() == [(0, 1), (1, 2), (2, 4), (4, 8)]
    assert list(P.leaf)[:8] == [7, 6, 5, 4, 3, 2, 1, 0]
    assert P.masks() == ((1 << 2) | (1 << 4) | (1 << 6) | (1 << 12), (1 << 1) | (1 << 2) | (1 << 4))
    with pytest.raises(ValueError):
        mvx.plan(mvx.COLL_ALLREDUCE, 16, 0, 1 << 20, 10, 102).masks()
