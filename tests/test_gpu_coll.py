"""GPU parity of the collectives: device results == the reference schedule.

Virtual communicators (p ranks' buffers on the one GPU of the test box) run
exactly the per-rank plans the RCCL path runs, so every combine order is
checked on the device; the RCCL transport itself is exercised with a
one-rank communicator here and by the multi-GPU bench on the driver's node.
The expected values come from oracle/coll_sim.c, which replays the
reference's message schedule (intra_fns_new.c) with the oracle op.
"""
import numpy as np
import pytest

import mvxtest as T

pytestmark = pytest.mark.gpu

CASES = [(102, 10), (100, 10), (101, 11), (111, 17), (110, 18), (105, 8), (103, 6), (108, 4), (111, 20),
         (110, 21), (102, 24), (109, 3), (102, 12), (100, 12), (111, 22)]
SIZES = [1, 7, 10, 1000, 2047, 2048, 4097, 16385, 70001, 140001]


def _run(mvx, comm, coll, p, sends, n_or_cnts, dtype, op, root=0):
    import torch
    ds = [T.to_dev(s) for s in sends]
    if coll == "rs":
        cnts = n_or_cnts
        drs = [torch.zeros(max(c, 1) * sends[0].dtype.itemsize, dtype=torch.uint8, device="cuda") for c in cnts]
        r, rcs = comm.reduce_scatter_multi(ds, drs, cnts, dtype, op)
    elif coll == "ar":
        drs = [torch.zeros(sends[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r, rcs = comm.allreduce_multi(ds, drs, n_or_cnts, dtype, op)
    else:
        drs = [torch.zeros(sends[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r, rcs = comm.reduce_multi(ds, drs, n_or_cnts, dtype, op, root)
    assert r == 0
    return [T.from_dev(x) for x in drs], rcs


@pytest.fixture(scope="module")
def comms(mvx):
    cs = {p: mvx.Comm.local_ranks(p, 0) for p in range(1, 9)}
    yield cs
    for c in cs.values():
        c.free()


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("op,dtype", CASES)
def test_allreduce_matches_reference_schedule(mvx, oracle, comms, p, op, dtype):
    for n in SIZES:
        sends = [T.rand_vec(dtype, n, 1000 * p + 17 * r + n) for r in range(p)]
        got, rcs = _run(mvx, comms[p], "ar", p, sends, n, dtype, op)
        refs = [np.zeros_like(sends[0]) for _ in range(p)]
        rref = oracle.allreduce([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], n, dtype, op)
        assert rcs == rref
        for r in range(p):
            T.assert_same(op, dtype, got[r], refs[r], typemap_only=True)


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("op,dtype", CASES)
def test_reduce_matches_reference_schedule(mvx, oracle, comms, p, op, dtype):
    for n in SIZES[::2]:
        for root in sorted({0, p - 1, p // 2}):
            sends = [T.rand_vec(dtype, n, 99 * p + 7 * r + n + root) for r in range(p)]
            got, rcs = _run(mvx, comms[p], "red", p, sends, n, dtype, op, root)
            refs = [np.zeros_like(sends[0]) for _ in range(p)]
            rref = oracle.reduce([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], n, dtype,
                                 op, root)
            assert rcs == rref
            T.assert_same(op, dtype, got[root], refs[root], typemap_only=True)


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("op,dtype", CASES)
def test_scan_matches_reference_schedule(mvx, oracle, comms, p, op, dtype):
    import torch
    for n in (1, 10, 5000, 70001):
        sends = [T.rand_vec(dtype, n, 7 * p + 3 * r + n) for r in range(p)]
        ds = [T.to_dev(s) for s in sends]
        drs = [torch.zeros(sends[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r, rcs = comms[p].scan_multi(ds, drs, n, dtype, op)
        assert r == 0
        refs = [np.zeros_like(sends[0]) for _ in range(p)]
        rref = oracle.scan([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], n, dtype, op)
        assert rcs == rref
        for q in range(p):
            T.assert_same(op, dtype, T.from_dev(drs[q]), refs[q], typemap_only=True)


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("op,dtype", CASES)
def test_reduce_scatter_matches_reference_schedule(mvx, oracle, comms, p, op, dtype):
    for base in (0, 1, 3, 500, 20000, 70000):
        cnts = [max(0, base + (r % 3) - 1) for r in range(p)]
        total = sum(cnts)
        sends = [T.rand_vec(dtype, max(total, 1), 31 * p + r + base) for r in range(p)]
        got, rcs = _run(mvx, comms[p], "rs", p, sends, cnts, dtype, op)
        refs = [np.zeros(max(c, 1), sends[0].dtype) for c in cnts]
        rref = oracle.reduce_scatter([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], cnts,
                                     dtype, op)
        assert rcs == rref
        for r in range(p):
            if cnts[r]:
                T.assert_same(op, dtype, got[r][: cnts[r] * sends[0].dtype.itemsize], refs[r][: cnts[r]],
                              typemap_only=True)


def test_nan_roles_survey_a3(mvx, oracle, comms):
    """SURVEY.md A.3, measured on the reference: MAX with a NaN on rank 1 at
    p = 4 -- recursive doubling (small): only rank 1 ends with NaN;
    Rabenseifner (large): exactly the block rank 1 owns is NaN on every rank."""
    p = 4
    for n, expect in ((8, "doubling"), (65536, "rabenseifner")):
        sends = [np.full(n, 1.0, np.float32) for _ in range(p)]
        sends[1][:] = np.nan
        got, rcs = _run(mvx, comms[p], "ar", p, sends, n, 10, 100)
        vals = [g.view(np.float32) for g in got]
        if expect == "doubling":
            assert [bool(np.isnan(v).all()) for v in vals] == [False, True, False, False]
        else:
            for v in vals:
                assert int(np.isnan(v).sum()) == n // 4
                assert np.array_equal(np.isnan(v), np.isnan(vals[0]))


def test_error_semantics_survey_a5(mvx, comms):
    """BAND on FLOAT -> 329 on every rank that calls the op;
    p = 1 never calls it -> 0; count 0 -> 0."""
    import torch
    x = [torch.zeros(64, device="cuda") for _ in range(8)]
    y = [torch.zeros(64, device="cuda") for _ in range(8)]
    r, rcs = comms[4].allreduce_multi(x[:4], y[:4], 64, 10, 105)
    assert r == 0 and rcs == [329] * 4
    r, rcs = comms[1].allreduce_multi(x[:1], y[:1], 64, 10, 105)
    assert rcs == [0]
    r, rcs = comms[4].allreduce_multi(x[:4], y[:4], 0, 10, 105)
    assert rcs == [0] * 4
    r, rcs = comms[4].reduce_multi(x[:4], y[:4], 64, 10, 105, 0)
    assert rcs[0] == 329
    r, rcs = comms[4].reduce_scatter_multi(x[:4], y[:4], [16] * 4, 10, 105)
    assert rcs == [329] * 4


def test_allreduce_c3_shape_8_ranks(mvx, oracle, comms):
    """Config 3's algorithm (p = 8 Rabenseifner, SUM f32) at 8 Mi elements
    per rank (virtual ranks share one GPU's HBM), bit-exact."""
    p, n = 8, 8 * 1024 * 1024
    sends = [np.empty(n, np.float32) for _ in range(p)]
    for r in range(p):
        oracle.fill(sends[r], n, 0, r)
    got, rcs = _run(mvx, comms[p], "ar", p, sends, n, 10, 102)
    refs = [np.zeros(n, np.float32) for _ in range(p)]
    oracle.allreduce([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], n, 10, 102)
    for r in range(p):
        assert np.array_equal(got[r].view(np.uint32), refs[r].view(np.uint32))


def test_rccl_single_rank_world(mvx, oracle):
    """The RCCL communicator path (mvx_comm_init) with one rank: blocking
    MPI_Allreduce / MPI_Reduce / MPI_Reduce_scatter on device and host
    buffers, and the reference's argument-error codes."""
    import os

    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
    comm = mvx.Comm.from_torch_distributed(0)
    n = 100000
    a = np.empty(n, np.float32)
    oracle.fill(a, n, 0, 0)
    da = torch.from_numpy(a).cuda()
    db = torch.zeros_like(da)
    assert mvx.MPI_Allreduce(da, db, n, 10, 102, comm) == 0
    assert np.array_equal(db.cpu().numpy(), a)
    hb = np.zeros(n, np.float32)
    assert mvx.MPI_Allreduce(a, hb, n, 10, 102, comm) == 0          # host buffers, staged
    assert np.array_equal(hb, a)
    hr = np.zeros(n, np.float32)
    assert mvx.MPI_Reduce(a, hr, n, 10, 100, 0, comm) == 0
    assert np.array_equal(hr, a)
    hs = np.zeros(n, np.float32)
    assert mvx.MPI_Reduce_scatter(a, hs, [n], 10, 102, comm) == 0
    assert np.array_equal(hs, a)
    hc = np.zeros(n, np.float32)
    assert mvx.MPI_Scan(a, hc, n, 10, 102, comm) == 0
    assert np.array_equal(hc, a)
    dc = torch.zeros_like(da)
    assert comm.scan_async(da, dc, n, 10, 102) == 0
    torch.cuda.synchronize()
    assert np.array_equal(dc.cpu().numpy(), a)
    # argument errors: reference order and codes
    code = mvx.MPI_Allreduce(da, da, n, 10, 102, comm)
    assert mvx.error_class(code) == mvx.MPI_ERR_BUFFER and (code >> 6) & 0x7f == 7
    assert mvx.error_class(mvx.MPI_Allreduce(da, db, -1, 10, 102, comm)) == mvx.MPI_ERR_COUNT
    assert mvx.MPI_Allreduce(da, db, n, 99, 102, comm) == 3 | (5 << 6)
    assert mvx.MPI_Allreduce(da, db, n, 10, 77, comm) == mvx.MPI_ERR_OP
    assert mvx.MPI_Allreduce(da, db, 0, 10, 77, comm) == 0
    assert mvx.error_class(mvx.MPI_Reduce(da, db, n, 10, 102, 3, comm)) == mvx.MPI_ERR_ROOT
    # p = 1: the op is never called, so an undefined pair is not an error
    assert mvx.MPI_Allreduce(da, db, n, 10, 105, comm) == 0
    # async path on torch's stream
    db.zero_()
    assert comm.allreduce_async(da, db, n, 10, 102) == 0
    torch.cuda.synchronize()
    assert np.array_equal(db.cpu().numpy(), a)
    # the variant each call ran: p = 1 moves nothing between ranks
    assert comm.last_exchange() == -1
    comm.free()
    # mvx_comm_abort (ncclCommAbort) with a call still queued: the handle is
    # released at once and the queued work completes; a fresh communicator
    # on the same group works
    comm = mvx.Comm.from_torch_distributed(0)
    db.zero_()
    assert comm.allreduce_async(da, db, n, 10, 102) == 0
    assert comm.abort() == 0
    torch.cuda.synchronize()
    assert np.array_equal(db.cpu().numpy(), a)
    comm = mvx.Comm.from_torch_distributed(0)
    db.zero_()
    assert mvx.MPI_Allreduce(da, db, n, 10, 102, comm) == 0
    assert np.array_equal(db.cpu().numpy(), a)
    comm.free()


def _full_size(mvx, oracle, comms, coll, p, n_elems, dtype, op, dist, cnts=None):
    """Every rank of a BASELINE config at its full size, on one GPU's HBM."""
    import torch
    npdt = T.np_dtype(dtype)
    sends = []
    for r in range(p):
        a = np.empty(n_elems, npdt)
        oracle.fill(a, n_elems, dist, r)
        sends.append(a)
    ds = [torch.from_numpy(a.view(np.uint8)).cuda() for a in sends]
    if coll == "rs":
        drs = [torch.empty(c * npdt.itemsize, dtype=torch.uint8, device="cuda") for c in cnts]
        r, rcs = comms[p].reduce_scatter_multi(ds, drs, cnts, dtype, op)
        refs = [np.zeros(c, npdt) for c in cnts]
        rref = oracle.reduce_scatter([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], cnts,
                                     dtype, op)
    else:
        drs = [torch.empty(n_elems * npdt.itemsize, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r, rcs = comms[p].allreduce_multi(ds, drs, n_elems, dtype, op)
        refs = [np.zeros(n_elems, npdt) for _ in range(p)]
        rref = oracle.allreduce([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], n_elems,
                                dtype, op)
    assert r == 0 and rcs == rref == [0] * p
    del ds
    for q in range(p):
        got = T.from_dev(drs[q])
        T.assert_same(op, dtype, got, refs[q], typemap_only=True)
        drs[q] = None
    torch.cuda.empty_cache()


def test_c3_full_size_allreduce_sum_f32_8x256mib(mvx, oracle, comms):
    """Config 3 at full size: 8 ranks x 256 MiB MPI_FLOAT MPI_SUM,
    Rabenseifner order, bit-exact on every rank."""
    _full_size(mvx, oracle, comms, "ar", 8, 64 << 20, 10, 102, 0)


def test_c4_full_size_reduce_scatter_band_int64_4x1gib(mvx, oracle, comms):
    """Config 4 at full size: 4 ranks x 1 GiB MPI_LONG MPI_BAND (pairwise
    chain), recvcnts 33554432 x 4, bit-exact."""
    n = 1 << 27
    _full_size(mvx, oracle, comms, "rs", 4, n, 8, 105, 2, cnts=[n // 4] * 4)


@pytest.mark.parametrize("dist", [3, 4])
def test_c5_full_size_allreduce_maxloc_float_int_8x64mi(mvx, oracle, comms, dist):
    """Config 5 at full size: 8 ranks x 64 Mi MPI_FLOAT_INT pairs MPI_MAXLOC
    with many ties (v = u % 1024), bit-exact, on both SURVEY.md 8(d) index
    choices: loc = rank (3, every tie is settled by the min-loc rule across
    ranks) and loc = rank*n + i (4)."""
    _full_size(mvx, oracle, comms, "ar", 8, 64 << 20, 17, 111, dist)


@pytest.mark.parametrize("p", [5, 6, 7])
@pytest.mark.parametrize("op,dtype", [(102, 10), (105, 8)])
def test_large_pairwise_reduce_scatter_five_to_seven_ranks(mvx, oracle, comms, p, op, dtype):
    """The pairwise Reduce_scatter at p = 5..7 with blocks large enough for a
    non-temporal combine: each rank's p-leaf chain runs the 8-leaf chain
    body with a run-time leaf count (k_chain_body, MVX_CHAIN_RT) -- against
    the reference schedule's replay."""
    E = 4 if dtype == 10 else 8
    blk = (16 << 20) // E
    cnts = [blk] * p
    sends = [T.rand_vec(dtype, blk * p, 4242 + 13 * p + r) for r in range(p)]
    got, rcs = _run(mvx, comms[p], "rs", p, sends, cnts, dtype, op)
    assert mvx.last_kernel_symbol().startswith("k_chain_body<"), mvx.last_kernel_symbol()
    refs = [np.zeros(c, sends[0].dtype) for c in cnts]
    rref = oracle.reduce_scatter([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in refs], cnts,
                                 dtype, op)
    assert rcs == rref
    for r in range(p):
        T.assert_same(op, dtype, got[r][: cnts[r] * E], refs[r], typemap_only=True)
