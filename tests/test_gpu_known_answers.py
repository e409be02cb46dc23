"""GPU: the device path against the reference's own known answers.

Every answer the reference's tests assert for this path
(tests/golden/known_answers.json, from examples/test/coll/allred.c,
redscat.c, coll12.c, redtst.c, shortint.c, scantst.c) is fed straight to the
MI355X path and compared with the stored expected values -- not with the
oracle -- in both device flavours (ch_shmem collops, and the _SMP_ collops
whose count-10 calls take the leader path), from device buffers and from
host buffers (the staged pipeline), and through the 1-rank RCCL
communicator where the reference test runs at size 1.

Config 1 (BASELINE.json configs[0]): MPI_Reduce MPI_SUM MPI_INT of 1 MiB
(262,144 elements) at p = 2, root 0, host buffers -- the binomial tree
(intra_fns_new.c:4876-4954) through the staged path, checked against the
closed form of SURVEY.md 8(d) and against the oracle's replay.
"""
import numpy as np
import pytest

import golden_util as G
import mvxtest as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comms(mvx):
    cs = {}
    for p in (1, 2, 4):
        plain = mvx.Comm.local_ranks(p, 0)
        smp = mvx.Comm.local_ranks(p, 0)
        assert smp.set_tuning(mvx.smp_tuning()) == 0
        cs[p] = {"ch_shmem": plain, "smp": smp}
    yield cs
    for d in cs.values():
        for c in d.values():
            c.free()


def _bufs(inputs, where):
    import torch
    if where == "device":
        sends = [T.to_dev(x) for x in inputs]
        recvs = [torch.zeros(inputs[0].nbytes, dtype=torch.uint8, device="cuda") for _ in inputs]
    else:
        sends = [T.clone(x).view(np.uint8) for x in inputs]
        recvs = [np.zeros(inputs[0].nbytes, np.uint8) for _ in inputs]
    return sends, recvs


def _host(r):
    return r if isinstance(r, np.ndarray) else T.from_dev(r)


ALLRED = list(G.allred_items())


@pytest.mark.parametrize("flavour", ["ch_shmem", "smp"])
@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("item", ALLRED, ids=lambda it: "%s-%s-p%d-%d" % (it[1], it[2], it[3], it[0]))
def test_allred_c_known_answers_on_device(mvx, comms, flavour, where, item):
    """allred.c (examples/test/coll/allred.c): every (op, type) case at the
    communicator sizes it runs, every rank's result == the test's answer."""
    k, tname, oname, size, inputs, expected = item
    sends, recvs = _bufs(inputs, where)
    r, rcs = comms[size][flavour].allreduce_multi(sends, recvs, len(expected), G.handle(tname), G.handle(oname))
    assert r == 0 and rcs == [0] * size
    for q in range(size):
        got = _host(recvs[q]).view(expected.dtype)
        assert G.equal(got, expected), (k, tname, oname, size, q, got, expected)


def _run_other(mvx, comm, c, where):
    t, o, size = G.handle(c["type"]), G.handle(c["op"]), c["size"]
    ins = [G.to_array(x, c["type"]) for x in c["inputs"]]
    if c["coll"] == "reduce_scatter":
        import torch
        if where == "device":
            sends = [T.to_dev(x) for x in ins]
            recvs = [torch.zeros(max(n, 1) * ins[0].itemsize, dtype=torch.uint8, device="cuda") for n in c["recvcnts"]]
        else:
            sends = [T.clone(x).view(np.uint8) for x in ins]
            recvs = [np.zeros(max(n, 1) * ins[0].itemsize, np.uint8) for n in c["recvcnts"]]
        r, rcs = comm.reduce_scatter_multi(sends, recvs, c["recvcnts"], t, o)
        assert r == 0 and rcs == [0] * size
        for q in range(size):
            exp = G.to_array(c["expected"][q], c["type"])
            assert G.equal(_host(recvs[q]).view(exp.dtype)[: exp.size], exp), (c["test"], q)
        return
    sends, recvs = _bufs(ins, where)
    if c["coll"] == "scan":
        r, rcs = comm.scan_multi(sends, recvs, c["count"], t, o)
    elif c["coll"] == "allreduce":
        r, rcs = comm.allreduce_multi(sends, recvs, c["count"], t, o)
    else:
        r, rcs = comm.reduce_multi(sends, recvs, c["count"], t, o, c["root"])
    assert r == 0 and rcs == [0] * size
    if c["coll"] == "reduce":
        exp = G.to_array(c["expected_root"], c["type"])
        assert G.equal(_host(recvs[c["root"]]).view(exp.dtype), exp), c["test"]
    else:
        for q in range(size):
            exp = G.to_array(c["expected"][q], c["type"])
            assert G.equal(_host(recvs[q]).view(exp.dtype), exp), (c["test"], q)


@pytest.mark.parametrize("flavour", ["ch_shmem", "smp"])
@pytest.mark.parametrize("where", ["device", "host"])
def test_other_reference_tests_on_device(mvx, flavour, where):
    """redscat.c, coll12.c, redtst.c, shortint.c, scantst.c known answers."""
    done = 0
    cache = {}
    for c in G.load()["other"]:
        size = c["size"]
        if size not in cache:
            cache[size] = mvx.Comm.local_ranks(size, 0)
            if flavour == "smp":
                assert cache[size].set_tuning(mvx.smp_tuning()) == 0
        _run_other(mvx, cache[size], c, where)
        done += 1
    for cm in cache.values():
        cm.free()
    assert done >= 10


def test_size_one_known_answers_through_rccl(mvx):
    """The reference tests that also run at size 1 (redscat.c at np = 1),
    through the RCCL communicator's blocking MPI_* entry points, device and
    host buffers."""
    import os

    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
    comm = mvx.Comm.from_torch_distributed(0)
    ones = [c for c in G.load()["other"] if c["size"] == 1]
    assert ones
    for c in ones:
        t, o = G.handle(c["type"]), G.handle(c["op"])
        x = G.to_array(c["inputs"][0], c["type"])
        for where in ("device", "host"):
            if where == "device":
                s, r = T.to_dev(x), torch.zeros(max(x.nbytes, 16), dtype=torch.uint8, device="cuda")
            else:
                s, r = T.clone(x).view(np.uint8), np.zeros(max(x.nbytes, 16), np.uint8)
            if c["coll"] == "reduce_scatter":
                rc = mvx.MPI_Reduce_scatter(s, r, c["recvcnts"], t, o, comm)
                exp = G.to_array(c["expected"][0], c["type"])
            elif c["coll"] == "reduce":
                rc = mvx.MPI_Reduce(s, r, c["count"], t, o, c["root"], comm)
                exp = G.to_array(c["expected_root"], c["type"])
            elif c["coll"] == "scan":
                rc = mvx.MPI_Scan(s, r, c["count"], t, o, comm)
                exp = G.to_array(c["expected"][0], c["type"])
            else:
                rc = mvx.MPI_Allreduce(s, r, c["count"], t, o, comm)
                exp = G.to_array(c["expected"][0], c["type"])
            assert rc == 0
            assert G.equal(_host(r)[: exp.nbytes].view(exp.dtype), exp), (c["test"], where)
    comm.free()


def test_c1_reduce_sum_int_1mib_p2_host_buffers(mvx, oracle):
    """Config 1 at its workload: 2 ranks, MPI_Reduce(MPI_SUM, MPI_INT,
    262,144 elements, root 0) from host buffers through the staged pipeline;
    a[i] = i*(rank+1) so the root's answer is 3i."""
    n, p = 262144, 2
    comm = mvx.Comm.local_ranks(p, 0)
    sends = [(np.arange(n, dtype=np.int64) * (r + 1)).astype(np.int32) for r in range(p)]
    recvs = [np.zeros(n, np.int32) for _ in range(p)]
    assert mvx.algorithm(mvx.COLL_REDUCE, p, n, mvx.MPI_INT) == mvx.ALG_BINOMIAL
    r, rcs = comm.reduce_multi(sends, recvs, n, mvx.MPI_INT, mvx.MPI_SUM, 0)
    assert r == 0 and rcs == [0, 0]
    assert np.array_equal(recvs[0], (np.arange(n, dtype=np.int64) * 3).astype(np.int32))
    ref = [np.zeros(n, np.int32) for _ in range(p)]
    assert oracle.reduce([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in ref], n,
                         mvx.MPI_INT, mvx.MPI_SUM, 0) == [0, 0]
    assert np.array_equal(recvs[0], ref[0])
    assert not recvs[1].any()            # a non-root recvbuf is not written
    # the same through the oracle's random inputs, both roots
    for root in (0, 1):
        S = [T.rand_vec(mvx.MPI_INT, n, 5 + r) for r in range(p)]
        R = [np.zeros(n, np.int32) for _ in range(p)]
        r, rcs = comm.reduce_multi(S, R, n, mvx.MPI_INT, mvx.MPI_SUM, root)
        assert r == 0 and rcs == [0, 0]
        ref = [np.zeros(n, np.int32) for _ in range(p)]
        oracle.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in ref], n, mvx.MPI_INT,
                      mvx.MPI_SUM, root)
        assert np.array_equal(R[root], ref[root])
    comm.free()


@pytest.mark.parametrize("flavour", ["ch_shmem", "smp"])
@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("p", [2, 4])
def test_successive_calls_do_not_interfere(mvx, comms, flavour, where, p):
    """examples/test/coll/allred2.c (MPI_Allreduce of one int, alternating
    +-10, checked after every call: 10 * size) and allredmany.c (MPI_Allreduce
    of the double 10.0, repeated) -- back-to-back calls on one communicator
    reuse its staging pool, so a stale slot would show here."""
    import torch
    comm = comms[p][flavour]

    def bufs(vals, dt):
        if where == "device":
            return ([torch.tensor([v], dtype=dt, device="cuda") for v in vals],
                    [torch.zeros(1, dtype=dt, device="cuda") for _ in vals])
        npdt = np.int32 if dt == torch.int32 else np.float64
        return [np.array([v], npdt) for v in vals], [np.zeros(1, npdt) for _ in vals]

    for i in range(200):                                      # allred2.c, MAX_LOOP 1000
        v = 10 if i & 1 else -10
        s, r = bufs([v] * p, torch.int32)
        rc, rcs = comm.allreduce_multi(s, r, 1, mvx.MPI_INT, mvx.MPI_SUM)
        assert rc == 0 and rcs == [0] * p
        for x in r:
            got = int(x.cpu()[0]) if where == "device" else int(x[0])
            assert got == v * p, (i, got)
    s, r = bufs([10.0] * p, torch.float64)
    for i in range(200):                                      # allredmany.c, 10000 calls
        rc, rcs = comm.allreduce_multi(s, r, 1, mvx.MPI_DOUBLE, mvx.MPI_SUM)
        assert rc == 0
    for x in r:
        got = float(x.cpu()[0]) if where == "device" else float(x[0])
        assert got == 10.0 * p


@pytest.mark.parametrize("flavour", ["ch_shmem", "smp"])
@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("p", [2, 4])
def test_coll8_coll13_known_answers(mvx, comms, flavour, where, p):
    """examples/test/coll/coll8.c: MPI_Reduce of data = rank to root 0 with
    MPI_SUM (sum of ranks), MPI_MIN (0) and MPI_MAX (size - 1); coll13.c:
    MPI_Allreduce(MPI_SUM) of every rank's MPI_Alltoall status (0 -> 0)."""
    import torch
    comm = comms[p][flavour]

    def bufs(vals):
        if where == "device":
            return ([torch.tensor([v], dtype=torch.int32, device="cuda") for v in vals],
                    [torch.full((1,), -100, dtype=torch.int32, device="cuda") for _ in vals])
        return [np.array([v], np.int32) for v in vals], [np.full(1, -100, np.int32) for _ in vals]

    def val(x):
        return int(x.cpu()[0]) if where == "device" else int(x[0])

    for op, want in ((mvx.MPI_SUM, sum(range(p))), (mvx.MPI_MIN, 0), (mvx.MPI_MAX, p - 1)):
        s, r = bufs(list(range(p)))
        rc, rcs = comm.reduce_multi(s, r, 1, mvx.MPI_INT, op, 0)
        assert rc == 0 and rcs == [0] * p
        assert val(r[0]) == want, (op, val(r[0]))
        assert all(val(x) == -100 for x in r[1:])         # non-roots: recvbuf untouched
    s, r = bufs([0] * p)
    rc, rcs = comm.allreduce_multi(s, r, 1, mvx.MPI_INT, mvx.MPI_SUM)
    assert rc == 0 and all(val(x) == 0 for x in r)
