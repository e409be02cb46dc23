"""GPU: the executor around the kernels.

* Host buffers (MPI user buffers live in host memory, allreduce.c:57-92):
  the staged pipeline slices every rank's plan (mvx_exec.c mvxi_plan_slice) and
  overlaps host copies, H2D, the collective and D2H.  Pageable, page-locked
  and mixed host/device buffers, several slices per call, against the
  oracle's replay of the reference schedule.
* Communicators above 8 ranks: combines of more than 8 leaves run as groups
  of <= 8-leaf launches (predefined ops) or step by step (user ops); p = 9,
  16, 33 against the replay (binomial Reduce, pairwise / halving
  Reduce_scatter, Rabenseifner at pof2 = 16 / 32, Scan on ranks >= 8).
* The reference's argument-test order (mpi_error.h:403-405, 524-526).
"""
import numpy as np
import pytest

import mvxtest as T
import uops

pytestmark = pytest.mark.gpu


def _oracle_coll(oracle, coll, S, R, n_or_cnts, dtype, op, root=0):
    s8 = [s.view(np.uint8) for s in S]
    r8 = [r.view(np.uint8) for r in R]
    if coll == "ar":
        return oracle.allreduce(s8, r8, n_or_cnts, dtype, op)
    if coll == "red":
        return oracle.reduce(s8, r8, n_or_cnts, dtype, op, root)
    if coll == "scan":
        return oracle.scan(s8, r8, n_or_cnts, dtype, op)
    return oracle.reduce_scatter(s8, r8, n_or_cnts, dtype, op)


def _call(comm, coll, sends, recvs, n_or_cnts, dtype, op, root=0):
    if coll == "ar":
        return comm.allreduce_multi(sends, recvs, n_or_cnts, dtype, op)
    if coll == "red":
        return comm.reduce_multi(sends, recvs, n_or_cnts, dtype, op, root)
    if coll == "scan":
        return comm.scan_multi(sends, recvs, n_or_cnts, dtype, op)
    return comm.reduce_scatter_multi(sends, recvs, n_or_cnts, dtype, op)


def _pinned_like(a):
    import torch
    t = torch.empty(a.nbytes, dtype=torch.uint8, pin_memory=True)
    t.numpy()[:] = np.ascontiguousarray(a).view(np.uint8)
    return t


def _to_np(buf):
    import torch
    if isinstance(buf, torch.Tensor):
        if buf.is_cuda:
            torch.cuda.synchronize()
        return buf.cpu().numpy()
    return buf


@pytest.mark.parametrize("where", ["pageable", "pinned", "send_dev_recv_host", "send_host_recv_dev"])
@pytest.mark.parametrize("p", [1, 3, 8])
@pytest.mark.parametrize("coll", ["ar", "red", "rs", "scan"])
def test_staged_pipeline_matches_reference(mvx, oracle, where, p, coll):
    import torch
    comm = mvx.Comm.local_ranks(p, 0)
    try:
        for dtype, op in ((10, 102), (17, 111), (8, 105)):
            E = mvx.dtype_info(dtype)[0]
            n = (3 << 20) // E + 17          # several 16 MiB slices at p = 8, a ragged tail
            cnts = [n // p + (r % 3) for r in range(p)] if coll == "rs" else None
            tot = sum(cnts) if cnts else n
            S = [T.rand_vec(dtype, tot, 100 * p + r + dtype) for r in range(p)]
            rb = [(cnts[r] if cnts else n) * E for r in range(p)]
            if where == "pageable":
                sends = [T.clone(s).view(np.uint8) for s in S]
                recvs = [np.zeros(max(b, 1), np.uint8) for b in rb]
            elif where == "pinned":
                sends = [_pinned_like(s) for s in S]
                recvs = [torch.zeros(max(b, 1), dtype=torch.uint8, pin_memory=True) for b in rb]
            elif where == "send_dev_recv_host":
                sends = [T.to_dev(s) for s in S]
                recvs = [np.zeros(max(b, 1), np.uint8) for b in rb]
            else:
                sends = [T.clone(s).view(np.uint8) for s in S]
                recvs = [torch.zeros(max(b, 1), dtype=torch.uint8, device="cuda") for b in rb]
            root = p - 1
            r, rcs = _call(comm, coll, sends, recvs, cnts if cnts else n, dtype, op, root)
            assert r == 0
            R0 = [np.zeros(max(cnts[q] if cnts else n, 1), S[0].dtype) for q in range(p)]
            rref = _oracle_coll(oracle, coll, S, R0, cnts if cnts else n, dtype, op, root)
            assert rcs == rref
            for q in range(p):
                if coll == "red" and q != root:
                    assert not _to_np(recvs[q]).any()    # non-root recvbuf untouched
                    continue
                cnt = cnts[q] if cnts else n
                T.assert_same(op, dtype, _to_np(recvs[q])[: cnt * E], R0[q][:cnt], typemap_only=True)
    finally:
        comm.free()


WIDE_CASES = [(102, 10), (100, 10), (111, 17), (105, 8), (110, 18)]


@pytest.fixture(scope="module")
def wide(mvx):
    cs = {p: mvx.Comm.local_ranks(p, 0) for p in (9, 16, 33)}
    yield cs
    for c in cs.values():
        c.free()


@pytest.mark.parametrize("p", [9, 16, 33])
@pytest.mark.parametrize("op,dtype", WIDE_CASES)
def test_wide_communicators(mvx, oracle, wide, p, op, dtype):
    import torch
    comm = wide[p]
    E = mvx.dtype_info(dtype)[0]
    for coll, n in (("ar", 7), ("ar", 20000), ("red", 9), ("red", 20000), ("rs", 3), ("rs", 9000), ("scan", 300)):
        cnts = [n + (r % 2) for r in range(p)] if coll == "rs" else None
        tot = sum(cnts) if cnts else n
        S = [T.rand_vec(dtype, tot, 7 * p + r + n) for r in range(p)]
        ds = [T.to_dev(s) for s in S]
        drs = [torch.zeros(max((cnts[q] if cnts else n), 1) * E, dtype=torch.uint8, device="cuda")
               for q in range(p)]
        root = p // 2
        r, rcs = _call(comm, coll, ds, drs, cnts if cnts else n, dtype, op, root)
        assert r == 0
        R0 = [np.zeros(max(cnts[q] if cnts else n, 1), S[0].dtype) for q in range(p)]
        rref = _oracle_coll(oracle, coll, S, R0, cnts if cnts else n, dtype, op, root)
        assert rcs == rref, (coll, n)
        ranks = [root] if coll == "red" else range(p)
        for q in ranks:
            cnt = cnts[q] if cnts else n
            T.assert_same(op, dtype, T.from_dev(drs[q])[: cnt * E], R0[q][:cnt], typemap_only=True)


@pytest.mark.parametrize("device_fn", [False, True], ids=["host_fn", "device_fn"])
@pytest.mark.parametrize("name,commute", [("mix", 0), ("affine", 0), ("fsum", 1)])
def test_wide_user_ops(mvx, oracle, wide, name, commute, device_fn):
    import torch
    if device_fn:
        rc, h = mvx.op_create_device(uops.dev_fn(name), commute)
    else:
        rc, h = mvx.MPI_Op_create(uops.host_fn(name), commute)
    assert rc == 0
    assert oracle.user_op_set(250, uops.host_fn(name), commute) == 0
    dt = uops.UOPS[name][0]
    try:
        for p in (9, 16):
            comm = wide[p]
            for coll, n in (("ar", 33), ("red", 33), ("rs", 200), ("scan", 33)):
                cnts = [n + (r % 2) for r in range(p)] if coll == "rs" else None
                tot = sum(cnts) if cnts else n
                S = [uops.rand_for(name, tot, 31 * p + r) for r in range(p)]
                E = S[0].itemsize
                ds = [T.to_dev(s) for s in S]
                drs = [torch.zeros((cnts[q] if cnts else n) * E, dtype=torch.uint8, device="cuda") for q in range(p)]
                r, rcs = _call(comm, coll, ds, drs, cnts if cnts else n, dt, h, 1)
                assert r == 0 and rcs == [0] * p
                R0 = [np.zeros(cnts[q] if cnts else n, S[0].dtype) for q in range(p)]
                _oracle_coll(oracle, coll, S, R0, cnts if cnts else n, dt, 250, 1)
                for q in ([1] if coll == "red" else range(p)):
                    assert T.bytes_equal(T.from_dev(drs[q]), R0[q]), (name, p, coll, q)
    finally:
        mvx.MPI_Op_free(h)


def test_argument_test_order(mvx):
    """MPIR_TEST_COUNT and MPIR_TEST_ALIAS both run; each failure advances
    the error ring, and the later test's code is returned (allreduce.c:76-77
    count then alias; reduce.c:82-83 and scan.c alias then count).
    MPI_BOTTOM (NULL) never aliases (mpi_error.h:524-526)."""
    import torch
    comm = mvx.Comm.local_ranks(2, 0)
    x = torch.zeros(16, device="cuda")
    h = comm.handle
    assert mvx.MPI_Allreduce(0, 0, 0, 10, 102, h) == 0
    assert mvx.MPI_Reduce(0, 0, 0, 10, 102, 0, h) == 0
    assert mvx.MPI_Scan(0, 0, 0, 10, 102, h) == 0
    a = mvx.MPI_Allreduce(x, x, -1, 10, 102, h)
    b = mvx.MPI_Allreduce(x, x, -1, 10, 102, h)
    assert a & 63 == mvx.MPI_ERR_BUFFER and (a >> 6) & 0x7f == 7     # alias wins (tested last)
    assert (b >> 13) - (a >> 13) == 2                                  # two setmsg calls per call
    c = mvx.MPI_Reduce(x, x, -1, 10, 102, 0, h)
    assert c & 63 == mvx.MPI_ERR_COUNT                                 # count tested last
    assert (c >> 13) - (b >> 13) == 2
    d = mvx.MPI_Scan(x, x, -1, 10, 102, h)
    assert d & 63 == mvx.MPI_ERR_COUNT
    e = mvx.MPI_Reduce_scatter(x, x, [1, 1], 10, 102, h)
    assert e & 63 == mvx.MPI_ERR_BUFFER and (e >> 13) - (d >> 13) == 1
    comm.free()


@pytest.mark.parametrize("slices", [2, 3, 5])
@pytest.mark.parametrize("p", [2, 3, 4, 8, 9])
def test_pipelined_exchange_matches_reference(mvx, oracle, slices, p):
    """MVX_EXCH_PIPE: slice t's exchange while slice t-1 combines on a
    second stream, then one unsliced distribution group on every rank (a
    non-root Reduce's temporary result included: it is kept whole in one
    shared temporary); loopback transport here, the RCCL
    executor's phase code -- same bits as the reference schedule for every
    collective, role-sensitive ops included."""
    import torch
    comm = mvx.Comm.local_ranks(p, 0)
    assert comm.set_exchange(mvx.EXCH_PIPE, slices) == 0
    assert comm.get_exchange() == (mvx.EXCH_PIPE, slices)
    try:
        for op, dtype in ((102, 10), (100, 10), (111, 17), (105, 8)):
            E = mvx.dtype_info(dtype)[0]
            for coll, n in (("ar", 5), ("ar", 300001), ("red", 200003), ("rs", 70001), ("scan", 50000)):
                cnts = [n // p + (r % 3) for r in range(p)] if coll == "rs" else None
                tot = sum(cnts) if cnts else n
                S = [T.rand_vec(dtype, tot, 13 * p + r + n) for r in range(p)]
                ds = [T.to_dev(s) for s in S]
                drs = [torch.zeros(max(cnts[q] if cnts else n, 1) * E, dtype=torch.uint8, device="cuda")
                       for q in range(p)]
                root = p - 1
                r, rcs = _call(comm, coll, ds, drs, cnts if cnts else n, dtype, op, root)
                assert r == 0
                R0 = [np.zeros(max(cnts[q] if cnts else n, 1), S[0].dtype) for q in range(p)]
                rref = _oracle_coll(oracle, coll, S, R0, cnts if cnts else n, dtype, op, root)
                assert rcs == rref
                for q in ([root] if coll == "red" else range(p)):
                    cnt = cnts[q] if cnts else n
                    T.assert_same(op, dtype, T.from_dev(drs[q])[: cnt * E], R0[q][:cnt], typemap_only=True)
    finally:
        comm.free()


@pytest.mark.parametrize("mode", ["p2p", "pipe"])
def test_phase_timing(mvx, mode):
    """mvx_comm_set_phase_timing: events around phases A / B / C of a device
    call; the pipelined variant (overlapping phases) reports the total only.
    Timing does not change the result."""
    import torch
    p, n = 4, 1 << 22
    comm = mvx.Comm.local_ranks(p, 0)
    try:
        if mode == "pipe":
            assert comm.set_exchange(mvx.EXCH_PIPE, 4) == 0
        with pytest.raises(RuntimeError):
            comm.phase_times()               # nothing timed yet
        S = [T.rand_vec(10, n, 77 + r) for r in range(p)]
        ds = [T.to_dev(s) for s in S]
        outs = []
        for timed in (False, True):
            assert comm.set_phase_timing(timed) == 0
            dr = [torch.zeros(n * 4, dtype=torch.uint8, device="cuda") for _ in range(p)]
            r, rcs = comm.allreduce_multi(ds, dr, n, 10, 102)
            assert r == 0 and rcs == [0] * p
            outs.append([T.from_dev(x) for x in dr])
        ph = comm.phase_times()
        assert ph["total"] > 0
        if mode == "p2p":
            assert ph["A"] > 0 and ph["B"] > 0 and ph["C"] > 0
            assert ph["A"] + ph["B"] + ph["C"] <= ph["total"] * 1.01 + 1e-3
        else:
            assert ph["A"] is None and ph["B"] is None and ph["C"] is None
        for a, b in zip(*outs):
            assert np.array_equal(a, b)
        assert comm.set_phase_timing(False) == 0
    finally:
        comm.free()


@pytest.mark.parametrize("n", [262145, 2097153, 786433])
@pytest.mark.parametrize("p", [1, 2])
@pytest.mark.parametrize("coll", ["ar", "red", "rs", "scan"])
def test_pageable_ragged_sizes(mvx, oracle, n, p, coll):
    """Pageable host buffers whose byte size divided by the copy pool's
    threads falls on a 4 KiB boundary with a remainder (1 MiB + 4 B,
    8 MiB + 4 B, 3 MiB + 4 B of floats): the bounce copies carry every byte
    (a split that rounded down dropped the last bytes % threads bytes)."""
    comm = mvx.Comm.local_ranks(p, 0)
    try:
        dtype, op, E = 10, 102, 4
        cnts = [n] * p if coll == "rs" else None
        tot = n * p if cnts else n
        S = [T.rand_vec(dtype, tot, 31 * n + r) for r in range(p)]
        sends = [T.clone(s).view(np.uint8) for s in S]
        recvs = [np.zeros(n * E, np.uint8) for _ in range(p)]
        r, rcs = _call(comm, coll, sends, recvs, cnts if cnts else n, dtype, op, 0)
        assert r == 0
        R0 = [np.zeros(n, S[0].dtype) for _ in range(p)]
        assert rcs == _oracle_coll(oracle, coll, S, R0, cnts if cnts else n, dtype, op, 0)
        for q in ([0] if coll == "red" else range(p)):
            T.assert_same(op, dtype, recvs[q], R0[q], typemap_only=True)
    finally:
        comm.free()


def test_two_communicators_interleaved(mvx, oracle):
    """Executor state is per communicator (mvx_work: staging pool, slice
    plans, rank tables): two communicators issuing stream-ordered calls on
    two streams, interleaved and in flight together -- a PIPE one (p = 4,
    3 slices) and a P2P one (p = 3) -- each get the reference's bits."""
    import torch
    ca, cb = mvx.Comm.local_ranks(4, 0), mvx.Comm.local_ranks(3, 0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        assert ca.set_exchange(mvx.EXCH_PIPE, 3) == 0
        jobs = []
        for it in range(4):
            for comm, p, st, coll, n in ((ca, 4, sa, "ar", 300001 + it), (cb, 3, sb, "rs", 90001 + it)):
                cnts = [n // p + (r % 2) for r in range(p)] if coll == "rs" else None
                tot = sum(cnts) if cnts else n
                S = [T.rand_vec(10, tot, 71 * it + 7 * p + r) for r in range(p)]
                ds = [T.to_dev(s) for s in S]
                drs = [torch.zeros(max(cnts[q] if cnts else n, 1) * 4, dtype=torch.uint8, device="cuda")
                       for q in range(p)]
                torch.cuda.synchronize()          # inputs written before the other streams read them
                r = _call_on(comm, coll, ds, drs, cnts if cnts else n, st)
                assert r[0] == 0, r
                jobs.append((coll, p, S, drs, cnts if cnts else n, ds))
        torch.cuda.synchronize()
        for coll, p, S, drs, nc, _ in jobs:
            R0 = [np.zeros(max(nc[q] if coll == "rs" else nc, 1), np.float32) for q in range(p)]
            rref = _oracle_coll(oracle, coll, S, R0, nc, 10, 102)
            assert rref == [0] * p
            for q in range(p):
                cnt = nc[q] if coll == "rs" else nc
                T.assert_same(102, 10, T.from_dev(drs[q])[: cnt * 4], R0[q][:cnt], typemap_only=True)
    finally:
        ca.free()
        cb.free()


def _call_on(comm, coll, sends, recvs, n_or_cnts, stream):
    if coll == "ar":
        return comm.allreduce_multi(sends, recvs, n_or_cnts, 10, 102, stream)
    return comm.reduce_scatter_multi(sends, recvs, n_or_cnts, 10, 102, stream)


def test_two_communicators_from_two_threads(mvx, oracle):
    """Blocking calls on two communicators from two host threads at once
    (each communicator's calls stay on one thread, as MPI orders them)."""
    import threading
    import torch
    comms = [mvx.Comm.local_ranks(4, 0), mvx.Comm.local_ranks(2, 0)]
    assert comms[0].set_exchange(mvx.EXCH_PIPE, 4) == 0
    errors, done = [], []

    def worker(w):
        try:
            torch.cuda.set_device(0)
            comm, p = comms[w], (4, 2)[w]
            for it in range(5):
                n = 200003 + 1000 * it + w
                S = [T.rand_vec(10, n, 1000 * w + 10 * it + r) for r in range(p)]
                ds = [T.to_dev(s) for s in S]
                drs = [torch.zeros(n * 4, dtype=torch.uint8, device="cuda") for _ in range(p)]
                torch.cuda.synchronize()
                r, rcs = _call(comm, "ar", ds, drs, n, 10, 102)
                if r != 0:
                    errors.append((w, it, r))
                    return
                R0 = [np.zeros(n, np.float32) for _ in range(p)]
                _oracle_coll(oracle, "ar", S, R0, n, 10, 102)
                for q in range(p):
                    T.assert_same(102, 10, T.from_dev(drs[q])[: n * 4], R0[q], typemap_only=True)
            done.append(w)
        except Exception as e:            # reported below
            errors.append((w, repr(e)[:300]))

    th = [threading.Thread(target=worker, args=(w,)) for w in range(2)]
    try:
        for t in th:
            t.start()
        for t in th:
            t.join(120)
        assert not any(t.is_alive() for t in th), "a worker did not finish"
        assert not errors and sorted(done) == [0, 1], errors
    finally:
        for c in comms:
            c.free()
