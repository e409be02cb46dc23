"""CPU: the oracle's user-op replays (MPI_Op_create; permanent == 0 and the
noncommutative branches of intra_fns_new.c / intra_scan.c).

Pinned by the reference's own user-op tests (examples/test/coll/coll9.c,
coll10.c, coll11.c, scantst.c, longuser.c: their checks are restated here),
and by algebra: for an associative op the rank-ordered product is what every
algorithm must produce -- except the noncommutative pairwise
Reduce_scatter, whose reference order (6487-6498) is checked literally.
"""
import numpy as np
import pytest

import uops

H = 230   # oracle handles used here


def _reg(oracle, name, commute=None, h=H):
    c = uops.UOPS[name][1] if commute is None else commute
    assert oracle.user_op_set(h, uops.host_fn(name), c) == 0
    return h


def _run(oracle, coll, sends, count, dtype, op, root=0, cnts=None):
    p = len(sends)
    if coll == "rs":
        recvs = [np.zeros(max(c, 1), sends[0].dtype) for c in cnts]
        rc = oracle.reduce_scatter([s.view(np.uint8) for s in sends], [r.view(np.uint8) for r in recvs], cnts,
                                   dtype, op)
    else:
        recvs = [np.zeros_like(sends[0]) for _ in range(p)]
        f = {"ar": oracle.allreduce, "scan": oracle.scan}.get(coll)
        if f:
            rc = f([s.view(np.uint8) for s in sends], [r.view(np.uint8) for r in recvs], count, dtype, op)
        else:
            rc = oracle.reduce([s.view(np.uint8) for s in sends], [r.view(np.uint8) for r in recvs], count, dtype,
                               op, root)
    assert rc == [0] * p
    return recvs


@pytest.mark.parametrize("p", range(1, 9))
def test_reference_user_op_tests(oracle, p):
    # coll9.c: Reduce with commutative addem to root 0 = sum of ranks
    h = _reg(oracle, "addem")
    data = [np.array([r], np.int32) for r in range(p)]
    assert _run(oracle, "red", data, 1, 6, h, 0)[0][0] == sum(range(p))
    # coll10.c: noncommutative assoc, root size-1: rank order, no BAD_ANSWER
    h = _reg(oracle, "assoc")
    assert _run(oracle, "red", data, 1, 6, h, p - 1)[p - 1][0] != 100000
    # coll11.c / scantst.c: Scan with addem = prefix sums; with assoc no BAD
    h = _reg(oracle, "addem")
    got = _run(oracle, "scan", data, 1, 6, h)
    assert [int(g[0]) for g in got] == [sum(range(r + 1)) for r in range(p)]
    h = _reg(oracle, "assoc")
    got = _run(oracle, "scan", data, 1, 6, h)
    assert all(g[0] != 100000 for g in got)
    # longuser.c: Allreduce with a user add on doubles, sizes 1 .. 65536
    h = _reg(oracle, "add_f64")
    n = 1
    while n < 100000:
        ins = [np.full(n, 1.0 if r & 1 else -1.0) for r in range(p)]
        got = _run(oracle, "ar", ins, n, 11, h)
        exp = -1.0 if p & 1 else 0.0
        assert all((g == exp).all() for g in got), n
        n *= 2


def _compose(xs):
    """rank-ordered product of affine maps, x0 first: in composed after inout."""
    acc = np.array(xs[0], np.uint64)
    for x in xs[1:]:
        a1, b1 = acc & np.uint64(0xffffffff), acc >> np.uint64(32)
        a2, b2 = x & np.uint64(0xffffffff), x >> np.uint64(32)
        acc = ((a1 * a2) & np.uint64(0xffffffff)) | (((a2 * b1 + b2) & np.uint64(0xffffffff)) << np.uint64(32))
    return acc


@pytest.mark.parametrize("p", range(1, 9))
def test_noncommutative_associative_orders(oracle, p):
    """Affine maps: Allreduce, Reduce (any root), Scan and the short
    Reduce_scatter give the rank-ordered composition; the long (pairwise)
    Reduce_scatter gives the reference's own order (src < rank: acc = x_src
    then acc; else acc then x_src)."""
    h = _reg(oracle, "affine")
    n = 300
    xs = [uops.rand_for("affine", n, 10 + r) for r in range(p)]
    full = _compose(xs)
    for g in _run(oracle, "ar", xs, n, 9, h):
        assert np.array_equal(g, full)
    for root in range(p):
        assert np.array_equal(_run(oracle, "red", xs, n, 9, h, root)[root], full)
    got = _run(oracle, "scan", xs, n, 9, h)
    for r in range(p):
        assert np.array_equal(got[r], _compose(xs[: r + 1]))
    for per in (3, 40):   # 3*p*8 < 512 bytes: recursive doubling; 40*p*8 >= 512 from p = 2
        cnts = [per] * p
        xr = [uops.rand_for("affine", per * p, 50 + r) for r in range(p)]
        alg = oracle.algorithm(3, p, per * p, 9, h)
        got = _run(oracle, "rs", xr, 0, 9, h, cnts=cnts)
        for r in range(p):
            blk = [x[r * per:(r + 1) * per] for x in xr]
            if alg == oracle.ALG_RS_RECDBL:
                exp = _compose(blk)
            else:
                assert alg == oracle.ALG_RS_PAIRWISE
                exp = blk[r]
                for i in range(1, p):
                    src = (r - i) % p
                    exp = _compose([blk[src], exp]) if src < r else _compose([exp, blk[src]])
            assert np.array_equal(got[r][:per], exp), (per, r, alg)


def test_algorithm_choices_for_user_ops(oracle):
    hc = _reg(oracle, "addem", 1, 231)
    hn = _reg(oracle, "mix", 0, 232)
    for p in (2, 4, 8):
        assert oracle.algorithm(1, p, 1 << 20, 6, hc) == oracle.ALG_RECDBL     # permanent == 0
        assert oracle.algorithm(1, p, 1 << 20, 6, 102) == (oracle.ALG_RECDBL if p == 2   # coll_table -1
                                                           else oracle.ALG_RABENSEIFNER)
        assert oracle.algorithm(2, p, 1 << 20, 6, hc) == oracle.ALG_BINOMIAL
        assert oracle.algorithm(3, p, 1000, 6, hc) == oracle.ALG_RS_HALVING
        assert oracle.algorithm(3, p, 127, 7, hn) == oracle.ALG_RS_RECDBL      # 508 bytes
        assert oracle.algorithm(3, p, 128, 7, hn) == oracle.ALG_RS_PAIRWISE    # 512 bytes
