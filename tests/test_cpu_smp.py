"""CPU: the _SMP_ device flavour (intra_shmem_Reduce / intra_shmem_Allreduce).

MVAPICH's own devices (ch_gen2, ch_smp, ch_gen2_ud) are built with _SMP_ and
put intra_shmem_Reduce / intra_shmem_Allreduce in the collops table
(src/coll/intra_fns_new.c:293-310).  Below 1 KiB (Reduce) / 32 KiB
(Allreduce) a commutative op takes the leader path: rank 0 folds ranks
1 .. p-1 into a copy of its own vector in rank order (4992-5198, 5793-5940),
after a len = 0 call of the op on every rank that rejects an undefined
(op, type) everywhere -- p = 1 included.

Pinning: the reference's own known answers (examples/test/coll/allred.c and
siblings, count 10 -- the leader path in an _SMP_ build) against the oracle's
replay of that code (oracle/coll_sim.c), then every rank's libmvx plan
against the replay, NaN roles and user ops included, at and around every
threshold edge and knob.
"""
import numpy as np
import pytest

import golden_util as G
import mvxtest as T
import uops
from plan_exec import run_plans

ALLREDUCE, REDUCE = 1, 2


@pytest.fixture
def smp(oracle):
    oracle.smp_set(1)
    yield oracle
    oracle.smp_set(0)


@pytest.mark.parametrize("item", list(G.allred_items()), ids=lambda it: "%s-%s-p%d-%d" % (it[1], it[2], it[3], it[0]))
def test_allred_c_known_answers_smp_flavour(smp, item):
    """allred.c's closed-form answers hold for the leader path too."""
    k, tname, oname, size, inputs, expected = item
    recvs = [np.zeros_like(expected) for _ in range(size)]
    rc = smp.allreduce([x.view(np.uint8) for x in inputs], [r.view(np.uint8) for r in recvs], len(expected),
                       G.handle(tname), G.handle(oname))
    assert rc == [0] * size
    for r in range(size):
        assert G.equal(recvs[r], expected), (k, tname, oname, size, r)


def test_other_reference_tests_smp_flavour(smp):
    for c in G.load()["other"]:
        size, t, o = c["size"], G.handle(c["type"]), G.handle(c["op"])
        ins = [G.to_array(x, c["type"]) for x in c["inputs"]]
        if c["coll"] == "allreduce":
            recvs = [np.zeros_like(ins[0]) for _ in range(size)]
            rc = smp.allreduce([x.view(np.uint8) for x in ins], [r.view(np.uint8) for r in recvs], c["count"], t, o)
            for r in range(size):
                assert G.equal(recvs[r], G.to_array(c["expected"][r], c["type"])), c["test"]
            assert rc == [0] * size
        elif c["coll"] == "reduce":
            recvs = [np.zeros_like(ins[0]) for _ in range(size)]
            rc = smp.reduce([x.view(np.uint8) for x in ins], [r.view(np.uint8) for r in recvs], c["count"], t, o,
                            c["root"])
            assert G.equal(recvs[c["root"]], G.to_array(c["expected_root"], c["type"])), c["test"]
            assert rc == [0] * size


def test_leader_fold_is_the_rank_order_chain(smp):
    """Float SUM below 32 KiB: ((x0 + x1) + x2) + ... on every rank (not the
    recursive-doubling tree of the ch_shmem build)."""
    rng = np.random.default_rng(3)
    n = 1000
    for p in (2, 3, 4, 8):
        s = [(rng.standard_normal(n) * 10.0 ** rng.integers(-4, 4, n)).astype(np.float32) for _ in range(p)]
        r = [np.zeros(n, np.float32) for _ in range(p)]
        assert smp.allreduce([x.view(np.uint8) for x in s], [x.view(np.uint8) for x in r], n, 10, 102) == [0] * p
        exp = s[0].copy()
        for i in range(1, p):
            exp = exp + s[i]
        for q in range(p):
            assert np.array_equal(r[q], exp), (p, q)
    smp.smp_set(0)
    r0 = [np.zeros(n, np.float32) for _ in range(8)]
    smp.allreduce([x.view(np.uint8) for x in s], [x.view(np.uint8) for x in r0], n, 10, 102)
    assert not np.array_equal(r0[0], exp)       # the two flavours differ in the bits


def test_nan_roles_leader(smp):
    """MAX with a NaN on rank 1: the leader's accumulator is x0 (inout), an
    incoming NaN is dropped, so every rank gets 1.0 -- unlike the ch_shmem
    build's recursive doubling, where rank 1 keeps its NaN."""
    p, n = 4, 8
    s = [np.full(n, 1.0, np.float32) for _ in range(p)]
    s[1][:] = np.nan
    r = [np.zeros(n, np.float32) for _ in range(p)]
    smp.allreduce([x.view(np.uint8) for x in s], [x.view(np.uint8) for x in r], n, 10, 100)
    assert all(not np.isnan(v).any() for v in r)
    s[0][:] = np.nan
    smp.allreduce([x.view(np.uint8) for x in s], [x.view(np.uint8) for x in r], n, 10, 100)
    assert all(np.isnan(v).all() for v in r)


def test_error_semantics_smp(smp):
    """The len = 0 pre-check: BAND on FLOAT fails on every rank, p = 1 too
    (the ch_shmem build returns 0 at p = 1); count 0 -> 0."""
    x = [np.zeros(1 << 14, np.float32).view(np.uint8) for _ in range(4)]
    y = [np.zeros(1 << 14, np.float32).view(np.uint8) for _ in range(4)]
    assert smp.allreduce(x, y, 64, 10, 105) == [329] * 4
    assert smp.allreduce(x[:1], y[:1], 64, 10, 105) == [329]
    assert smp.reduce(x, y, 64, 10, 105, 2) == [329] * 4
    assert smp.reduce(x, y, 1 << 14, 10, 105, 2) == [329] * 4        # above the threshold too
    assert smp.allreduce(x, y, 0, 10, 105) == [0] * 4
    assert smp.reduce_scatter(x, y, [16] * 4, 10, 105) == [329] * 4  # Reduce_scatter is not shmem


CASES = [(102, 10), (100, 10), (101, 11), (103, 11), (111, 17), (110, 18), (105, 8), (102, 6), (108, 4),
         (110, 21), (111, 20), (102, 12), (100, 12), (111, 22), (103, 24)]


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("op,dtype", CASES)
def test_smp_allreduce_plans(mvx, smp, p, op, dtype):
    tun = mvx.smp_tuning()
    E = mvx.dtype_info(dtype)[0]
    thr = 1 << 15
    for n in sorted({1, 10, 333, max(thr // E - 1, 1), thr // E, thr // E + 1, 9000}):
        S = [T.rand_vec(dtype, n, 1000 * p + 17 * r + n) for r in range(p)]
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        rc = smp.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op)
        plans = [mvx.plan(mvx.COLL_ALLREDUCE, p, r, n, dtype, op, tuning=tun) for r in range(p)]
        assert (plans[0].alg == mvx.ALG_SMP_LEADER) == (n * E < thr)
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in range(p):
            T.assert_same(op, dtype, R1[r], R0[r], typemap_only=True)
        assert rc == [0] * p


@pytest.mark.parametrize("p", range(1, 9))
@pytest.mark.parametrize("op,dtype", CASES[::2])
def test_smp_reduce_plans(mvx, smp, p, op, dtype):
    tun = mvx.smp_tuning()
    E = mvx.dtype_info(dtype)[0]
    thr = 1 << 10
    for n in sorted({1, 7, max(thr // E - 1, 1), thr // E, thr // E + 1, 5000}):
        for root in sorted({0, 1 % p, p - 1}):
            S = [T.rand_vec(dtype, n, 77 * p + 13 * r + n + root) for r in range(p)]
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            smp.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op, root)
            plans = [mvx.plan(mvx.COLL_REDUCE, p, r, n, dtype, op, root, tuning=tun) for r in range(p)]
            assert (plans[0].alg == mvx.ALG_SMP_LEADER) == (n * E < thr)
            R1 = run_plans(plans, [s.view(np.uint8) for s in S],
                           [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
            T.assert_same(op, dtype, R1[root], R0[root], typemap_only=True)


@pytest.mark.parametrize("knobs,ok", [
    (dict(), True),
    (dict(disable_shmem_allreduce=1, disable_shmem_reduce=1), False),
    (dict(enable_shmem_collectives=0), False),
    (dict(shmem_coll_ok=0), False),
    (dict(shmem_coll_allreduce_threshold=4096, shmem_coll_reduce_threshold=64), True),
])
def test_knobs_choose_the_path(mvx, oracle, knobs, ok):
    """Every knob of 5849-5854 / 5066-5070, plan and replay side by side;
    the pre-check stays whatever the knobs say."""
    tun = mvx.smp_tuning(**knobs)
    okw = dict(enable=tun.enable_shmem_collectives, ok=tun.shmem_coll_ok, dis_red=tun.disable_shmem_reduce,
               dis_ar=tun.disable_shmem_allreduce, thr_red=tun.shmem_coll_reduce_threshold,
               thr_ar=tun.shmem_coll_allreduce_threshold)
    try:
        oracle.smp_set(1, **okw)
        for coll, n in ((ALLREDUCE, 100), (ALLREDUCE, 2000), (REDUCE, 10), (REDUCE, 200)):
            p = 4
            alg = mvx.algorithm(coll, p, n, 10, tuning=tun)
            thr = tun.shmem_coll_allreduce_threshold if coll == ALLREDUCE else tun.shmem_coll_reduce_threshold
            assert (alg == mvx.ALG_SMP_LEADER) == (ok and 4 * n < thr), (coll, n, alg)
            S = [T.rand_vec(10, n, 5 * r + n) for r in range(p)]
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            if coll == ALLREDUCE:
                rc = oracle.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, 10, 102)
            else:
                rc = oracle.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, 10, 102, 1)
            assert rc == [0] * p
            plans = [mvx.plan(coll, p, r, n, 10, 102, 1, tuning=tun) for r in range(p)]
            R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
            for r in (range(p) if coll == ALLREDUCE else [1]):
                T.assert_same(102, 10, R1[r], R0[r])
            assert all(P.calls_uop for P in [mvx.plan(coll, p, r, n, 10, 105, 1, tuning=tun) for r in range(p)])
    finally:
        oracle.smp_set(0)


def test_stride_is_the_reference_int_product(mvx):
    """`int stride = count*extent`: a vector of exactly 2 GiB wraps to a
    negative stride and takes the leader path, as in the reference."""
    tun = mvx.smp_tuning()
    assert mvx.algorithm(ALLREDUCE, 8, 1 << 29, 10, tuning=tun) == mvx.ALG_SMP_LEADER   # 2 GiB of float
    assert mvx.algorithm(ALLREDUCE, 8, (1 << 29) - 1, 10, tuning=tun) == mvx.ALG_RABENSEIFNER
    assert mvx.algorithm(ALLREDUCE, 8, 8191, 10, tuning=tun) == mvx.ALG_SMP_LEADER
    assert mvx.algorithm(ALLREDUCE, 8, 8192, 10, tuning=tun) == mvx.ALG_RABENSEIFNER
    # extent, not size: DOUBLE_INT is 16 bytes of extent, 12 of size
    assert mvx.algorithm(ALLREDUCE, 8, 2047, 18, tuning=tun) == mvx.ALG_SMP_LEADER
    assert mvx.algorithm(ALLREDUCE, 8, 2048, 18, tuning=tun) != mvx.ALG_SMP_LEADER
    # Reduce_scatter and Scan keep the plain algorithms
    assert mvx.algorithm(3, 8, 100, 10, tuning=tun) == mvx.ALG_RS_HALVING
    assert mvx.algorithm(4, 8, 100, 10, tuning=tun) == mvx.ALG_SCAN_RECDBL


@pytest.mark.parametrize("p", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("name,commute", [("mix", 1), ("mix", 0), ("fsum", 1), ("affine", 0)])
def test_smp_user_ops(mvx, smp, p, name, commute):
    """A commutative user op takes the leader path ((*uop)(x_i, acc), rank
    order); a noncommutative one falls through to intra_Allreduce /
    intra_Reduce with their noncommutative branches."""
    tun = mvx.smp_tuning()
    H = 240
    assert smp.user_op_set(H, uops.host_fn(name), commute) == 0
    dt = uops.UOPS[name][0]
    kind = 1 if commute else 2
    for n in (1, 50, 3000, 20000):
        S = [uops.rand_for(name, n, 11 * p + 7 * r + n) for r in range(p)]
        E = S[0].itemsize
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        smp.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dt, H)
        plans = [mvx.plan(ALLREDUCE, p, r, n, dt, H, opkind=kind, tuning=tun) for r in range(p)]
        assert (plans[0].alg == mvx.ALG_SMP_LEADER) == (bool(commute) and n * E < (1 << 15))
        R1 = run_plans(plans, [s.view(np.uint8) for s in S], [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
        for r in range(p):
            assert np.array_equal(R1[r].view(S[0].dtype), R0[r]), (n, r)
        for root in sorted({0, p - 1}):
            R0 = [np.zeros_like(S[0]) for _ in range(p)]
            smp.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dt, H, root)
            plans = [mvx.plan(REDUCE, p, r, n, dt, H, root, opkind=kind, tuning=tun) for r in range(p)]
            R1 = run_plans(plans, [s.view(np.uint8) for s in S],
                           [np.zeros(S[0].nbytes, np.uint8) for _ in range(p)])
            assert np.array_equal(R1[root].view(S[0].dtype), R0[root]), (n, root)


def test_tuning_from_env(mvx, monkeypatch):
    """initutil.c:230-293 knob parsing."""
    t = mvx.tuning_from_env(True)
    assert (t.smp, t.enable_shmem_collectives, t.shmem_coll_ok) == (1, 1, 1)
    assert (t.shmem_coll_reduce_threshold, t.shmem_coll_allreduce_threshold) == (1024, 32768)
    t = mvx.tuning_from_env(False)
    assert t.smp == 0
    monkeypatch.setenv("VIADEV_USE_SHMEM_ALLREDUCE", "0")
    monkeypatch.setenv("VIADEV_SHMEM_COLL_REDUCE_THRESHOLD", "4096")
    t = mvx.tuning_from_env(True)
    assert t.disable_shmem_allreduce == 1 and t.disable_shmem_reduce == 0
    assert t.shmem_coll_reduce_threshold == 4096
    monkeypatch.setenv("VIADEV_USE_BLOCKING", "1")
    t = mvx.tuning_from_env(True)
    assert t.enable_shmem_collectives == 0 and t.shmem_coll_ok == 0
    monkeypatch.setenv("VIADEV_SHMEM_COLL_ALLREDUCE_THRESHOLD", str(1 << 17))   # > max msg size (1 << 16)
    with pytest.raises(ValueError):
        mvx.tuning_from_env(True)
    monkeypatch.setenv("VIADEV_SHMEM_COLL_MAX_MSG_SIZE", str(1 << 18))
    assert mvx.tuning_from_env(True).shmem_coll_allreduce_threshold == 1 << 17
