"""GPU parity of the _SMP_ flavour (intra_shmem_Reduce / intra_shmem_Allreduce).

A virtual communicator switched to the _SMP_ collops (mvx_comm_set_tuning)
runs its leader-path plans on the device -- one exchange of whole vectors,
then the rank-order chain as one combine kernel -- and is compared with the
oracle's replay of the reference code (oracle/coll_sim.c, smp = 1).
"""
import numpy as np
import pytest

import mvxtest as T
import uops

pytestmark = pytest.mark.gpu

CASES = [(102, 10), (100, 10), (101, 11), (111, 17), (110, 18), (105, 8), (103, 6), (108, 4), (111, 20),
         (110, 21), (102, 24), (109, 3), (102, 12), (100, 12), (111, 22)]


@pytest.fixture(scope="module")
def smp_comms(mvx):
    cs = {}
    for p in range(1, 9):
        c = mvx.Comm.local_ranks(p, 0)
        assert c.set_tuning(mvx.smp_tuning()) == 0
        assert c.get_tuning().smp == 1
        cs[p] = c
    yield cs
    for c in cs.values():
        c.free()


@pytest.fixture
def smp(oracle):
    oracle.smp_set(1)
    yield oracle
    oracle.smp_set(0)


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("op,dtype", CASES)
def test_smp_allreduce_reduce_on_device(mvx, smp, smp_comms, p, op, dtype):
    import torch
    E = mvx.dtype_info(dtype)[0]
    for n in sorted({1, 10, 100, (1 << 10) // E, (1 << 15) // E - 1, (1 << 15) // E, 5000}):
        S = [T.rand_vec(dtype, n, 1000 * p + 17 * r + n) for r in range(p)]
        ds = [T.to_dev(s) for s in S]
        drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r, rcs = smp_comms[p].allreduce_multi(ds, drs, n, dtype, op)
        assert r == 0
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        rref = smp.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op)
        assert rcs == rref
        for q in range(p):
            T.assert_same(op, dtype, T.from_dev(drs[q]), R0[q], typemap_only=True)
        root = p - 1
        drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r, rcs = smp_comms[p].reduce_multi(ds, drs, n, dtype, op, root)
        assert r == 0
        R0 = [np.zeros_like(S[0]) for _ in range(p)]
        rref = smp.reduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dtype, op, root)
        assert rcs == rref
        T.assert_same(op, dtype, T.from_dev(drs[root]), R0[root], typemap_only=True)


def test_smp_error_semantics_on_device(mvx, smp_comms):
    """The len = 0 pre-check reports on every rank, p = 1 included."""
    import torch
    x = [torch.zeros(64, device="cuda") for _ in range(4)]
    y = [torch.zeros(64, device="cuda") for _ in range(4)]
    assert smp_comms[4].allreduce_multi(x, y, 64, 10, 105) == (0, [329] * 4)
    assert smp_comms[1].allreduce_multi(x[:1], y[:1], 64, 10, 105) == (0, [329])
    assert smp_comms[4].reduce_multi(x, y, 64, 10, 105, 3) == (0, [329] * 4)


@pytest.mark.parametrize("name,commute", [("mix", 1), ("fsum", 1), ("mix", 0)])
def test_smp_user_ops_on_device(mvx, smp, smp_comms, name, commute):
    import torch
    rc, h = mvx.MPI_Op_create(uops.host_fn(name), commute)
    assert rc == 0
    assert smp.user_op_set(250, uops.host_fn(name), commute) == 0
    dt = uops.UOPS[name][0]
    try:
        for p in (2, 3, 8):
            for n in (5, 3000):
                S = [uops.rand_for(name, n, 9 * p + r + n) for r in range(p)]
                drs = [torch.zeros(S[0].nbytes, dtype=torch.uint8, device="cuda") for _ in range(p)]
                r, rcs = smp_comms[p].allreduce_multi([T.to_dev(s) for s in S], drs, n, dt, h)
                assert r == 0 and rcs == [0] * p
                R0 = [np.zeros_like(S[0]) for _ in range(p)]
                smp.allreduce([s.view(np.uint8) for s in S], [x.view(np.uint8) for x in R0], n, dt, 250)
                for q in range(p):
                    assert np.array_equal(T.from_dev(drs[q]).view(S[0].dtype), R0[q]), (p, n, q)
    finally:
        assert mvx.MPI_Op_free(h)[0] == 0
