"""CPU: pin the oracle to the reference's own known answers.

The reference cannot be built here without its configure step (DESIGN.md
section 3), so the oracle (oracle/cpu_ops.c + oracle/coll_sim.c) is pinned by
every known-answer check the reference's tests make for this path
(tests/golden/known_answers.json, from examples/test/coll/*.c) and by the
reference outputs SURVEY.md Appendix A.3 / A.5 recorded.
"""
import numpy as np
import pytest

import golden_util as G


def test_fixture_covers_every_op_and_allred_case():
    d = G.load()
    cases = d["allred"]["cases"]
    assert len(cases) == 122
    assert {c["op"] for c in cases} == {"MPI_SUM", "MPI_PROD", "MPI_MAX", "MPI_MIN", "MPI_LAND", "MPI_LOR",
                                       "MPI_LXOR", "MPI_BAND", "MPI_BOR", "MPI_BXOR", "MPI_MAXLOC",
                                       "MPI_MINLOC"}


@pytest.mark.parametrize("item", list(G.allred_items()), ids=lambda it: "%s-%s-p%d-%d" % (it[1], it[2], it[3], it[0]))
def test_allred_c_known_answers(oracle, item):
    k, tname, oname, size, inputs, expected = item
    recvs = [np.zeros_like(expected) for _ in range(size)]
    rc = oracle.allreduce([x.view(np.uint8) for x in inputs], [r.view(np.uint8) for r in recvs], len(expected),
                          G.handle(tname), G.handle(oname))
    assert rc == [0] * size
    for r in range(size):
        assert G.equal(recvs[r], expected), (k, tname, oname, size, r, recvs[r], expected)


def test_other_reference_tests(oracle):
    for c in G.load()["other"]:
        size, t, o = c["size"], G.handle(c["type"]), G.handle(c["op"])
        ins = [G.to_array(x, c["type"]) for x in c["inputs"]]
        if c["coll"] == "reduce_scatter":
            recvs = [np.zeros(n, ins[0].dtype) for n in c["recvcnts"]]
            rc = oracle.reduce_scatter([x.view(np.uint8) for x in ins], [r.view(np.uint8) for r in recvs],
                                       c["recvcnts"], t, o)
            for r in range(size):
                assert G.equal(recvs[r], G.to_array(c["expected"][r], c["type"])), c["test"]
        elif c["coll"] == "scan":
            recvs = [np.zeros_like(ins[0]) for _ in range(size)]
            rc = oracle.scan([x.view(np.uint8) for x in ins], [r.view(np.uint8) for r in recvs], c["count"], t, o)
            for r in range(size):
                assert G.equal(recvs[r], G.to_array(c["expected"][r], c["type"])), c["test"]
        elif c["coll"] == "allreduce":
            recvs = [np.zeros_like(ins[0]) for _ in range(size)]
            rc = oracle.allreduce([x.view(np.uint8) for x in ins], [r.view(np.uint8) for r in recvs], c["count"], t, o)
            for r in range(size):
                assert G.equal(recvs[r], G.to_array(c["expected"][r], c["type"])), c["test"]
        else:
            recvs = [np.zeros_like(ins[0]) for _ in range(size)]
            rc = oracle.reduce([x.view(np.uint8) for x in ins], [r.view(np.uint8) for r in recvs], c["count"], t, o,
                               c["root"])
            assert G.equal(recvs[c["root"]], G.to_array(c["expected_root"], c["type"])), c["test"]
        assert rc == [0] * size


def test_survey_a5_error_semantics(oracle):
    """Reference outputs recorded in SURVEY.md A.5."""
    x = [np.zeros(64, np.float32).view(np.uint8) for _ in range(4)]
    y = [np.zeros(64, np.float32).view(np.uint8) for _ in range(4)]
    assert oracle.allreduce(x, y, 64, 10, 105) == [329] * 4      # BAND on FLOAT, p = 4
    assert oracle.reduce(x, y, 64, 10, 105, 0)[0] == 329
    assert oracle.reduce_scatter(x, y, [16] * 4, 10, 105) == [329] * 4
    assert oracle.allreduce(x[:1], y[:1], 64, 10, 105) == [0]    # p = 1: op never called
    assert oracle.allreduce(x, y, 0, 10, 105) == [0] * 4         # count = 0
    assert oracle.allreduce(x, y, 64, 10, 55) == [9] * 4         # invalid op handle


def test_survey_a3_nan_roles(oracle):
    """MAX with NaN on rank 1, p = 4."""
    p = 4
    for n, small in ((8, True), (65536, False)):
        s = [np.full(n, 1.0, np.float32) for _ in range(p)]
        s[1][:] = np.nan
        r = [np.zeros(n, np.float32) for _ in range(p)]
        oracle.allreduce([x.view(np.uint8) for x in s], [x.view(np.uint8) for x in r], n, 10, 100)
        if small:
            assert [bool(np.isnan(v).all()) for v in r] == [False, True, False, False]
            assert all(not np.isnan(v).any() for i, v in enumerate(r) if i != 1)
        else:
            for v in r:
                assert int(np.isnan(v).sum()) == 16384
            # the block newrank 1 owns after halving with distance 1, 2:
            # block bitrev(1) = 2 -> elements 32768..49151
            assert np.isnan(r[0][32768:49152]).all()


def test_survey_a3_combine_orders(oracle):
    """which float-SUM association each algorithm produces
    (tree-adjacent for Allreduce; halving tree / rotated chain for
    Reduce_scatter below / above 512 KiB)."""
    rng = np.random.default_rng(5)
    for p in (2, 4, 8):
        n = 1 << 20
        s = [(rng.standard_normal(n) * 10.0 ** rng.integers(-4, 4, n)).astype(np.float32) for _ in range(p)]
        r = [np.zeros(n, np.float32) for _ in range(p)]
        oracle.allreduce([x.view(np.uint8) for x in s], [x.view(np.uint8) for x in r], n, 10, 102)
        level = list(s)
        while len(level) > 1:
            level = [level[i] + level[i + 1] for i in range(0, len(level), 2)]
        assert np.array_equal(r[0], level[0]), p
    p = 4
    for total_bytes, kind in ((64 * 1024, "halving"), (1 << 20, "chain")):
        n = total_bytes // 4
        s = [(rng.standard_normal(n) * 10.0 ** rng.integers(-4, 4, n)).astype(np.float32) for _ in range(p)]
        cn = [n // p] * p
        r = [np.zeros(n // p, np.float32) for _ in range(p)]
        oracle.reduce_scatter([x.view(np.uint8) for x in s], [x.view(np.uint8) for x in r], cn, 10, 102)
        for rank in range(p):
            blk = [x[rank * (n // p):(rank + 1) * (n // p)] for x in s]
            if kind == "halving":
                # ((x_r + x_{r^2}) + (x_{r^1} + x_{r^3}))
                exp = (blk[rank] + blk[rank ^ 2]) + (blk[rank ^ 1] + blk[rank ^ 3])
            else:
                exp = blk[rank]
                for i in range(1, p):
                    exp = exp + blk[(rank - i) % p]
            assert np.array_equal(r[rank], exp), (kind, rank)
