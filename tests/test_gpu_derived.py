"""GPU parity on derived contiguous datatypes (MPI_Type_contiguous).

MAXLOC / MINLOC on count-2 contiguous pairs of INT, LONG, LONG_LONG_INT,
SHORT, CHAR, FLOAT, DOUBLE, LONG_DOUBLE (global_ops.c:1387-1503, 1625-1740)
run as device kernels over {value, loc} pairs of the base type (the x87 pair
through the integer x87 emulation); the collectives move count * extent bytes
per element and combine in the reference's order.  Expected values: the
oracle (oracle/cpu_ops.c, coll_sim.c) on the same handles.  Bit-exact.
"""
import numpy as np
import pytest

import derived_util as D
import mvxtest as T
import uops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comms(mvx):
    cs = {p: mvx.Comm.local_ranks(p, 0) for p in (1, 2, 3, 4, 8)}
    yield cs
    for c in cs.values():
        c.free()


@pytest.mark.parametrize("base", sorted(D.PAIR_BASES))
@pytest.mark.parametrize("op", [110, 111])
def test_pair_kernels(mvx, oracle, base, op):
    rc, h = D.make_both(mvx, oracle, 2, base)
    try:
        for n, shift in ((4099, 0), (1 << 18, 0), (777, 1)):
            a, b = D.rand_pairs(base, n + 1, 5 + n), D.rand_pairs(base, n + 1, 6 + n)
            da, db = T.to_dev(a), T.to_dev(b)
            E = a.dtype.itemsize
            assert mvx.op_apply(op, h, da.data_ptr() + shift * E, db.data_ptr(), n) == 0
            ref = T.clone(b)
            assert oracle.op(op, h, a[shift:].view(np.uint8), ref.view(np.uint8), n) == 0
            D.assert_pairs_same(T.from_dev(db), ref)
    finally:
        D.free_both(mvx, oracle, h)


@pytest.mark.parametrize("base", [6, 10, 11, 12, 1])
@pytest.mark.parametrize("shape", [0, 1])
def test_pair_combine(mvx, oracle, base, shape):
    from plan_exec import combine_cpu
    rc, h = D.make_both(mvx, oracle, 2, base)
    try:
        n = 3001
        for k in (3, 8):
            leaves = [D.rand_pairs(base, n, 40 + q) for q in range(k)]
            dst = T.to_dev(np.zeros_like(leaves[0]))
            assert mvx.op_combine(111, h, [T.to_dev(x) for x in leaves], dst, n, shape=shape) == 0
            ref = combine_cpu(111, h, leaves[0].dtype.itemsize, [x.view(np.uint8) for x in leaves], None, shape, n)
            D.assert_pairs_same(T.from_dev(dst), ref.view(leaves[0].dtype))
    finally:
        D.free_both(mvx, oracle, h)


@pytest.mark.parametrize("p", [2, 3, 4, 8])
@pytest.mark.parametrize("base,op", [(10, 111), (11, 110), (6, 111), (8, 110), (12, 111), (4, 110)])
def test_collectives_on_derived_pairs(mvx, oracle, comms, p, base, op):
    import torch
    rc, h = D.make_both(mvx, oracle, 2, base)
    try:
        for n in (5, 3000, 70001):
            S = [D.rand_pairs(base, n, 17 * p + r + n) for r in range(p)]
            sb = [s.view(np.uint8) for s in S]
            ds = [T.to_dev(s) for s in S]
            drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
            r, rcs = comms[p].allreduce_multi(ds, drs, n, h, op)
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            assert r == 0 and rcs == oracle.allreduce(sb, [x.view(np.uint8) for x in R0], n, h, op) == [0] * p
            for q in range(p):
                D.assert_pairs_same(T.from_dev(drs[q]), R0[q])
            root = p // 2
            drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
            r, rcs = comms[p].reduce_multi(ds, drs, n, h, op, root)
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            oracle.reduce(sb, [x.view(np.uint8) for x in R0], n, h, op, root)
            D.assert_pairs_same(T.from_dev(drs[root]), R0[root])
            cnts = [n // p + (q % 2) for q in range(p)]
            tot = sum(cnts)
            S = [D.rand_pairs(base, tot, 3 * p + r + n) for r in range(p)]
            E = S[0].itemsize
            drs = [torch.zeros(max(c, 1) * E, dtype=torch.uint8, device="cuda") for c in cnts]
            r, rcs = comms[p].reduce_scatter_multi([T.to_dev(s) for s in S], drs, cnts, h, op)
            R0 = [np.zeros(max(c, 1), S[0].dtype) for c in cnts]
            oracle.reduce_scatter([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], cnts, h, op)
            for q in range(p):
                D.assert_pairs_same(T.from_dev(drs[q])[: cnts[q] * E], R0[q][: cnts[q]])
    finally:
        D.free_both(mvx, oracle, h)


def test_undefined_op_and_user_op_on_derived(mvx, oracle, comms):
    """SUM on a derived type: 329 on every calling rank, data untouched;
    a user function over contig(3, MPI_UNSIGNED) through the executor."""
    import torch
    rc, h = D.make_both(mvx, oracle, 3, 7)
    rc2, hop = mvx.MPI_Op_create(uops.host_fn("mix3"), 0)
    assert oracle.user_op_set(250, uops.host_fn("mix3"), 0) == 0
    try:
        x = [torch.zeros(1200, dtype=torch.uint8, device="cuda") for _ in range(4)]
        y = [torch.zeros(1200, dtype=torch.uint8, device="cuda") for _ in range(4)]
        assert comms[4].allreduce_multi(x, y, 100, h, 102) == (0, [329] * 4)
        for p in (2, 3, 8):
            n = 501
            S = [np.random.default_rng(p + r).integers(0, 1 << 32, 3 * n, dtype=np.uint64).astype(np.uint32)
                 for r in range(p)]
            drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
            r, rcs = comms[p].allreduce_multi([T.to_dev(s) for s in S], drs, n, h, hop)
            assert r == 0 and rcs == [0] * p
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            oracle.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, h, 250)
            for q in range(p):
                assert np.array_equal(T.from_dev(drs[q]), R0[q].view(np.uint8)), (p, q)
    finally:
        assert mvx.MPI_Op_free(hop)[0] == 0
        D.free_both(mvx, oracle, h)
