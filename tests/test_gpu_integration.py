"""The MVAPICH collops shim (integration/intra_mvx.c) driving the GPU path.

One rank (the harness's MPI_COMM_WORLD, integration/check/harness.c); the
shim creates its libmvx twin over RCCL on first use.  Device buffers must go
to libmvx (the stand-in for MVAPICH's own path counts its calls), results
must be the reference's for one rank (recvbuf = sendbuf's type-map bytes,
bytes outside the type map untouched), the attribute's delete callback must
free the twin, and MVX_HOST_BUFFERS=1 must route host buffers to libmvx.
User functions must see the caller's datatype handle (mvx_type_set_handle).

Across processes (the harness's board world, RCCL over its socket transport
with the ranks sharing the GPU): rank 0 passes device buffers and the others
host buffers in the same call -- every rank must go to libmvx (the route is
agreed) and get the reference's bits; and a rank whose device cannot be used
(MVX_DEVICE_ID out of range) must make every rank's call fail, not hang.
"""
import ctypes

import numpy as np
import pytest

import uops
from test_cpu_integration import FLOAT, INT, DOUBLE, UB, MPI_SUM, UNSIGNED, Nodes, _lib, _world

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def shim(mvx):
    return _lib()


def _dev(a):
    import torch
    return torch.from_numpy(a.copy()).cuda()


def test_device_buffers_take_the_gpu_path(mvx, oracle, shim):
    import torch
    N = Nodes(shim, oracle)
    f = N.basic(FLOAT)
    s = np.arange(4096, dtype=np.float32) * 0.5
    before = shim.h_host_calls()
    for coll in ("ar", "red", "rs", "scan"):
        ds, dr = _dev(s), torch.zeros(4096, dtype=torch.float32, device="cuda")
        if coll == "ar":
            rc = shim.h_allreduce(ds.data_ptr(), dr.data_ptr(), 4096, f[1], MPI_SUM)
        elif coll == "red":
            rc = shim.h_reduce(ds.data_ptr(), dr.data_ptr(), 4096, f[1], MPI_SUM, 0)
        elif coll == "rs":
            cn = (ctypes.c_int * 1)(4096)
            rc = shim.h_reduce_scatter(ds.data_ptr(), dr.data_ptr(), cn, f[1], MPI_SUM)
        else:
            rc = shim.h_scan(ds.data_ptr(), dr.data_ptr(), 4096, f[1], MPI_SUM)
        assert rc == 0, coll
        assert np.array_equal(dr.cpu().numpy(), s), coll
    assert shim.h_host_calls() == before


def test_derived_types_and_user_ops(mvx, oracle, shim):
    """{int; hole; double; UB at 24} and a strided vector move packed: the
    holes and the tail stay as the caller left them (user op; one rank)."""
    N = Nodes(shim, oracle)
    i, d, ub = N.basic(INT), N.basic(DOUBLE), N.basic(UB)
    st = N.struct([1, 1, 1], [0, 8, 24], [i, d, ub])
    vec = N.vector(5, 1, 3, N.basic(UNSIGNED))
    uop = shim.h_op_create(1)
    rng = np.random.default_rng(5)
    for (oh, node), op, ext in ((st, uop, 24), (vec, uop, 52)):
        n = 777
        s = rng.integers(0, 256, n * ext, dtype=np.uint8)
        r0 = np.full(n * ext, 0x5C, np.uint8)
        ds, dr = _dev(s), _dev(r0)
        rc = shim.h_allreduce(ds.data_ptr(), dr.data_ptr(), n, node, op)
        ref = r0.copy()
        oracle.type_copy(ref, s, n, oh)
        assert rc == 0
        assert np.array_equal(dr.cpu().numpy(), ref)


def test_host_buffers_on_request(mvx, oracle, shim, monkeypatch):
    N = Nodes(shim, oracle)
    f = N.basic(FLOAT)
    s = np.arange(100000, dtype=np.float32)
    r = np.zeros_like(s)
    before = shim.h_host_calls()
    monkeypatch.setenv("MVX_HOST_BUFFERS", "1")
    assert shim.h_allreduce(s.ctypes.data, r.ctypes.data, s.size, f[1], MPI_SUM) == 0
    assert shim.h_host_calls() == before and np.array_equal(r, s)
    monkeypatch.delenv("MVX_HOST_BUFFERS")
    r[:] = 0
    assert shim.h_allreduce(s.ctypes.data, r.ctypes.data, s.size, f[1], MPI_SUM) == 0
    assert shim.h_host_calls() == before + 1 and np.array_equal(r, s)


def test_comm_free_releases_the_twin(mvx, oracle, shim):
    N = Nodes(shim, oracle)
    f = N.basic(FLOAT)
    s = _dev(np.ones(64, np.float32))
    r = _dev(np.zeros(64, np.float32))
    assert shim.h_allreduce(s.data_ptr(), r.data_ptr(), 64, f[1], MPI_SUM) == 0
    assert shim.h_comm_free_attrs(91) == 1          # the delete callback ran
    assert shim.h_comm_free_attrs(91) == 0
    r.zero_()
    assert shim.h_allreduce(s.data_ptr(), r.data_ptr(), 64, f[1], MPI_SUM) == 0   # re-created
    assert float(r.sum()) == 64.0


@pytest.mark.parametrize("where", ["device", "host"])
def test_user_function_sees_callers_handle(mvx, where):
    import torch
    rc, t = mvx.MPI_Type_contiguous(3, mvx.MPI_UNSIGNED)
    assert rc == 0 and mvx.MPI_Type_commit(t) == 0
    rc, op = mvx.MPI_Op_create(uops.host_fn("mix3"), 0)
    assert rc == 0
    comm = mvx.Comm.local_ranks(2, 0)
    last = ctypes.c_int.in_dll(uops.host_lib(), "uop_last_dt")
    try:
        for alias in (4242, t):
            assert mvx.type_set_handle(t, alias) == 0
            last.value = -1
            S = [np.arange(300, dtype=np.uint32) + r for r in range(2)]
            if where == "device":
                sends = [torch.from_numpy(x.view(np.int32)).cuda() for x in S]
                recvs = [torch.zeros(300, dtype=torch.int32, device="cuda") for _ in S]
            else:
                sends = [x.copy() for x in S]
                recvs = [np.zeros(300, np.uint32) for _ in S]
            r, rcs = comm.allreduce_multi(sends, recvs, 100, t, op)
            assert r == 0 and rcs == [0, 0]
            assert last.value == alias
    finally:
        mvx.type_set_handle(t, t)
        comm.free()
        mvx.MPI_Op_free(op)
        mvx.MPI_Type_free(t)


@pytest.mark.parametrize("np_", [2, 3])
def test_mixed_buffer_kinds_through_the_shim(mvx, np_):
    """Rank 0 device buffers, the other ranks host buffers, one call: the
    agreed route takes every rank to libmvx (the host ranks through its HBM
    mirrors), no rank runs MVAPICH's path, and every rank's recvbuf is the
    oracle's replay of the reference schedule bit for bit -- Allreduce,
    Reduce (root np-1), Reduce_scatter (ragged counts) and Scan."""
    for rep in _world(np_, "mixed", timeout=300):
        assert not rep["fails"], rep
        assert len(rep["calls"]) == 4
        for c in rep["calls"]:
            assert c["rc"] == 0 and c["host"] == 0, c
        # the first call agreed the route and created the twin (two MIN
        # agreements); later calls agree the route only
        assert rep["calls"][0]["agree"] == 3 and all(c["agree"] == 1 for c in rep["calls"][1:]), rep


def test_twin_creation_failure_on_one_rank_fails_every_rank(mvx):
    """Rank 1's device is unusable (MVX_DEVICE_ID=99): the creation agreement
    stops every rank before RCCL's collective init, so both ranks return
    MPI_ERR_OTHER within seconds, and keep returning it."""
    reps = _world(2, "fail", {1: {"MVX_DEVICE_ID": "99"}}, timeout=180)
    for rep in reps:
        assert len(rep["calls"]) == 4
        for c in rep["calls"]:
            assert c["rc"] == 15 and c["host"] == 0 and c["s"] < 30, (rep["rank"], c)


@pytest.mark.parametrize("np_", [2, 3])
def test_within_rank_kinds_through_the_shim(mvx, np_):
    """Buffer kinds mixed within a rank (round 5's regression: a rank with a
    device sendbuf and a host recvbuf was counted as device, the shim passed
    MVX_KINDS_DEVICE, and that rank failed alone while its peers waited in
    RCCL):
      Reduce with device sendbufs everywhere and a host recvbuf at the root;
      Allreduce with device send and host recv on every rank;
      Reduce_scatter with host send and device recv on rank 0 only;
      Reduce with device buffers everywhere (the non-roots' host recvbuf is
      never touched: the call is agreed all-device);
      Scan with device sendbufs and host recvbufs on all ranks but the last.
    Every rank's recvbuf is the oracle's replay bit for bit, at 1000 and
    300001 floats (the larger one in slices: MVX_SLICE_MIN_MIB=1)."""
    env = {"MVX_SLICE_MIN_MIB": "1", "MVX_SLICE_MIB": "1"}
    for rep in _world(np_, "kinds", {r: env for r in range(np_)}, timeout=300):
        assert not rep["fails"], rep
        assert len(rep["calls"]) == 10
        for c in rep["calls"]:
            assert c["rc"] == 0 and c["host"] == 0 and c["agree"] in (1, 3), c
        dd = [c for c in rep["calls"] if c["name"].startswith("reduce_dd")]
        assert all(c["route_all"][1] == 0 for c in dd), dd        # agreed all-device


def test_route_agreement_latency(mvx):
    """The per-call route agreement's cost: an 8-byte device
    Allreduce at p = 2 through the shim, agreed vs MVX_SHIM_ROUTE=local, the
    agreement over the harness's host transport (a shared-memory board).
    Both modes must return the right sum; the medians are reported."""
    reps = _world(2, "latency", timeout=300)
    for rep in reps:
        assert not rep["fails"], rep
        print("rank", rep["rank"], "median us per call", rep["latency_us"])
