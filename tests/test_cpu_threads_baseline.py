"""CPU: the threaded CPU baseline (oracle/cpu_coll.c) computes what the
reference's schedules compute.

BASELINE.md section 4 times the reference's collectives on p host cores;
oracle/cpu_coll.c runs the intra_fns_new.c schedules with one thread per
rank over shared memory.  Its results must equal coll_sim.c's lockstep replay
bit for bit, or the timed baseline would not be the reference's work.
"""
import numpy as np
import pytest

import mvxtest as T


def _bufs(p, n, dtype, seed):
    S = [T.rand_vec(dtype, n, seed + r) for r in range(p)]
    R = [np.zeros_like(S[0]) for _ in range(p)]
    W = [np.zeros(2 * n * S[0].itemsize + 64, np.uint8) for _ in range(p)]
    return S, R, W


@pytest.mark.parametrize("p", [1, 2, 4, 8])
@pytest.mark.parametrize("op,dtype", [(102, 10), (100, 10), (111, 17), (105, 8), (102, 6)])
def test_threaded_allreduce_equals_replay(oracle, p, op, dtype):
    for n in (5, 1000, 70001):
        S, R, W = _bufs(p, n, dtype, 10 * p + n)
        t = oracle.threads_coll(1, [s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R], W, n, dtype, op)
        assert t > 0
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        oracle.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op)
        for r in range(p):
            T.assert_same(op, dtype, R[r].view(np.uint8), R0[r], typemap_only=True)


@pytest.mark.parametrize("p", [2, 4, 8])
def test_threaded_reduce_binomial_equals_replay(oracle, p):
    n = 1000        # binomial regime at every p (<= 4096 bytes)
    for root in range(p):
        S, R, W = _bufs(p, n, 10, 3 * p + root)
        oracle.threads_coll(2, [s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R], W, n, 10, 102,
                            root=root)
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        oracle.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, 10, 102, root)
        T.assert_same(102, 10, R[root].view(np.uint8), R0[root])


@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("base", [100, 70000])          # halving / pairwise
def test_threaded_reduce_scatter_equals_replay(oracle, p, base):
    cnts = [base + (r % 2) for r in range(p)]
    tot = sum(cnts)
    for op, dtype in ((102, 10), (105, 8)):
        S, _, W = _bufs(p, tot, dtype, 7 * p + base)
        R = [np.zeros(c, S[0].dtype) for c in cnts]
        oracle.threads_coll(3, [s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R], W, 0, dtype, op,
                            recvcnts=cnts)
        R0 = [np.zeros(c, S[0].dtype) for c in cnts]
        oracle.reduce_scatter([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], cnts, dtype, op)
        for r in range(p):
            T.assert_same(op, dtype, R[r].view(np.uint8), R0[r])
