"""GPU: collectives with user-defined ops (MPI_Op_create and the device
extension mvx_op_create_device) against the oracle's replay of the
reference's user-op branches.

Virtual communicators (p ranks on one GPU) run the RCCL executor's phase
code; phase B calls the user function step by step in the plan's operand
roles (host MPI_User_function: on pinned host copies of the leaves; device
function: stream-ordered on HBM scratch).  The oracle calls the same C host
function (tests/user_ops.c); the device functions (tests/user_ops_dev.hip)
compute the same bits.  Bit-exact.
"""
import numpy as np
import pytest

import mvxtest as T
import uops

pytestmark = pytest.mark.gpu

CASES = [("mix", 0), ("mix", 1), ("affine", 0), ("fsum", 1), ("fsum", 0), ("addem", 1)]


@pytest.fixture(scope="module")
def comms(mvx):
    cs = {p: mvx.Comm.local_ranks(p, 0) for p in range(1, 9)}
    yield cs
    for c in cs.values():
        c.free()


def _ops(mvx, oracle, name, commute, device):
    """(product handle, oracle handle) for the op; the oracle always runs the
    host function."""
    if device:
        rc, h = mvx.op_create_device(uops.dev_fn(name), commute)
    else:
        rc, h = mvx.MPI_Op_create(uops.host_fn(name), commute)
    assert rc == 0 and h >= 200
    assert oracle.user_op_set(250, uops.host_fn(name), commute) == 0
    return h, 250


def _dev(x):
    return T.to_dev(x)


@pytest.mark.parametrize("device", [False, True], ids=["host_fn", "device_fn"])
@pytest.mark.parametrize("name,commute", CASES)
def test_user_op_collectives(mvx, oracle, comms, name, commute, device):
    import torch
    h, oh = _ops(mvx, oracle, name, commute, device)
    dt = uops.UOPS[name][0]
    try:
        for p in range(1, 9):
            c = comms[p]
            for n in (1, 5, 100, 4097):
                S = [uops.rand_for(name, n, 1000 * p + 7 * r + n) for r in range(p)]
                ds = [_dev(s) for s in S]
                sb = [s.view(np.uint8) for s in S]
                # Allreduce
                drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
                r, rcs = c.allreduce_multi(ds, drs, n, dt, h)
                assert r == 0 and rcs == [0] * p
                R0 = [np.zeros_like(S[0]) for _ in range(p)]
                oracle.allreduce(sb, [x.view(np.uint8) for x in R0], n, dt, oh)
                for q in range(p):
                    assert np.array_equal(T.from_dev(drs[q]).view(S[0].dtype), R0[q]), ("ar", p, n, q)
                # Reduce, two roots
                for root in sorted({0, p - 1}):
                    drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
                    r, rcs = c.reduce_multi(ds, drs, n, dt, h, root)
                    assert r == 0
                    R0 = [np.zeros_like(S[0]) for _ in range(p)]
                    oracle.reduce(sb, [x.view(np.uint8) for x in R0], n, dt, oh, root)
                    assert np.array_equal(T.from_dev(drs[root]).view(S[0].dtype), R0[root]), ("red", p, n, root)
                # Scan
                drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
                r, rcs = c.scan_multi(ds, drs, n, dt, h)
                assert r == 0
                R0 = [np.zeros_like(S[0]) for _ in range(p)]
                oracle.scan(sb, [x.view(np.uint8) for x in R0], n, dt, oh)
                for q in range(p):
                    assert np.array_equal(T.from_dev(drs[q]).view(S[0].dtype), R0[q]), ("scan", p, n, q)
            # Reduce_scatter: short (recursive doubling if noncommutative) and long
            for base in (1, 3, 2000):
                cnts = [base + (r % 2) for r in range(p)]
                tot = sum(cnts)
                S = [uops.rand_for(name, tot, 77 * p + r + base) for r in range(p)]
                E = S[0].itemsize
                drs = [torch.zeros(max(cn, 1) * E, dtype=torch.uint8, device="cuda") for cn in cnts]
                r, rcs = c.reduce_scatter_multi([_dev(s) for s in S], drs, cnts, dt, h)
                assert r == 0
                R0 = [np.zeros(max(cn, 1), S[0].dtype) for cn in cnts]
                oracle.reduce_scatter([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], cnts, dt, oh)
                for q in range(p):
                    got = T.from_dev(drs[q]).view(S[0].dtype)[: cnts[q]]
                    assert np.array_equal(got, R0[q][: cnts[q]]), ("rs", p, base, q)
    finally:
        assert mvx.MPI_Op_free(h)[0] == 0


def test_reference_user_op_tests_single_rank_world(mvx):
    """coll9.c / coll10.c / longuser.c on the RCCL world at p = 1 (the box
    has one GPU), host buffers as in the reference tests."""
    import os

    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1)
    comm = mvx.Comm.from_torch_distributed(0)
    rc, h = mvx.MPI_Op_create(uops.host_fn("addem"), 1)
    data = np.array([0], np.int32)
    out = np.full(1, -100, np.int32)
    assert mvx.MPI_Reduce(data, out, 1, 6, h, 0, comm) == 0 and out[0] == 0
    rc, ha = mvx.MPI_Op_create(uops.host_fn("assoc"), 0)
    out[:] = -100
    assert mvx.MPI_Reduce(data, out, 1, 6, ha, 0, comm) == 0 and out[0] == 0
    assert mvx.MPI_Scan(data, out, 1, 6, ha, comm) == 0 and out[0] == 0
    rc, hd = mvx.MPI_Op_create(uops.host_fn("add_f64"), 1)
    for n in (1, 2, 1024, 65536):
        ib = np.full(n, -1.0)
        ob = np.full(n, 100.0)
        assert mvx.MPI_Allreduce(ib, ob, n, 11, hd, comm) == 0 and (ob == -1.0).all()
    # a device function on device buffers: stream-ordered, no host copies
    rc, hm = mvx.op_create_device(uops.dev_fn("fsum"), 1)
    x = torch.randn(1 << 20, device="cuda")
    y = torch.zeros_like(x)
    assert comm.allreduce_async(x, y, x.numel(), 10, hm) == 0
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    for op in (h, ha, hd, hm):
        assert mvx.MPI_Op_free(op)[0] == 0
    comm.free()
