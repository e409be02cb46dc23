"""CPU: the drop-in boundary loads and exports what include/*.h declares,
and its host-side behaviour (registries, argument checks, op verdicts) is
the reference's.  No kernel is launched here."""
import ctypes
import os
import re

import pytest

import mvxtest as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECL = re.compile(r"^\s*(?:extern\s+)?(?:const\s+)?(?:int|void|char)\s*\*?\s*([A-Za-z_]\w*)\s*\(", re.M)


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(DECL.findall(text)) - {"MPI_User_function"})


@pytest.mark.parametrize("header,lib", [("mvx_hip.h", "hip"), ("mvx_coll.h", "coll")])
def test_every_declared_symbol_is_exported(mvx, header, lib):
    names = declared(header)
    assert len(names) >= (6 if lib == "hip" else 40)
    L = mvx.hip() if lib == "hip" else mvx.coll()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_embed_library_exports_only_mvx_names(mvx):
    """libmvx_embed.so (csrc/embed.map): every function include/mvx_embed.h
    declares, and no MPI_ / PMPI_ / MPIR_ symbol that could collide with the
    host MPI's own when linked into MVAPICH (integration/intra_mvx.c)."""
    import subprocess
    so = os.path.join(ROOT, "mvapich-cce_amd", "libmvx_embed.so")
    out = subprocess.check_output(["nm", "-D", "--defined-only", so], text=True)
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    names = declared("mvx_embed.h")
    assert len(names) >= 15
    assert set(names) <= syms, sorted(set(names) - syms)
    bad = sorted(x for x in syms if re.match(r"(P?MPI_|MPIR_)", x))
    assert not bad, bad
    assert all(x.startswith(("mvx_", "MVX_")) for x in syms if not x.startswith("_")), sorted(syms)[:20]


def test_collops_table_exported(mvx):
    assert ctypes.c_void_p.in_dll(mvx.coll(), "MVX_device_collops") is not None


def test_libraries_are_in_tree(mvx):
    for p in mvx.loaded_paths():
        assert os.path.exists(p) and p.startswith(os.path.join(ROOT, "mvapich-cce_amd"))


def test_op_support_matrix_matches_reference(mvx, oracle):
    """mvx_op_supported / mvx_op_apply's verdict == global_ops.c's switch
    (SURVEY.md Appendix B), the x87 long double types included."""
    for op in range(100, 112):
        for dtype in T.ALL_TYPES:
            ref = T.oracle_rc(oracle, op, dtype)
            verdict = mvx.hip().mvx_op_apply(op, dtype, None, None, 0, None)
            assert verdict == ref, (op, dtype)
            assert bool(mvx.hip().mvx_op_supported(op, dtype)) == (ref == 0)
            assert (dtype in mvx.DEFINED[op]) == (ref == 0), (op, dtype)
    assert mvx.hip().mvx_op_apply(99, 10, None, None, 0, None) == mvx.MPI_ERR_OP


def test_dtype_extents(mvx, oracle):
    for dtype in T.ALL_TYPES:
        e, s = mvx.dtype_info(dtype)
        oe, os_ = oracle.dtype_info(dtype)
        assert (e, s) == (oe, os_), dtype
        assert mvx.hip().mvx_dtype_extent(dtype) == e
        assert mvx.NP_DTYPE[dtype].itemsize == e


def test_op_create_free_semantics(mvx):
    """MPI_Op_create / MPI_Op_free (opcreate.c:62-76, opfree.c:51-82)."""
    rc, op = mvx.MPI_Op_create(lambda a, b, n, t: None, 1)
    assert rc == 0 and op >= 200
    rc, newop = mvx.MPI_Op_free(op)
    assert rc == 0 and newop == mvx.MPI_OP_NULL
    rc, _ = mvx.MPI_Op_free(mvx.MPI_OP_NULL)
    assert rc == 9 | (3 << 6)                      # MPI_ERR_OP | MPIR_ERR_OP_NULL
    rc, _ = mvx.MPI_Op_free(mvx.MPI_SUM)
    assert rc == 12 | (13 << 6)                    # MPI_ERR_ARG | MPIR_ERR_PERM_OP
    assert mvx.error_class(rc) == mvx.MPI_ERR_ARG


def test_null_communicator_codes(mvx):
    """MPIR_TEST_MPI_COMM / MPIR_TEST_DTYPE run before anything touches the
    device (mpid/ch2/comm.h:130-135, datatype.h:64-68)."""
    assert mvx.MPI_Allreduce(0, 0, 1, 10, 102, 12345) == 5 | (3 << 6)
    assert mvx.MPI_Reduce(0, 0, 1, 10, 102, 0, 12345) == 5 | (3 << 6)
    assert mvx.MPI_Reduce_scatter(0, 0, [1], 10, 102, 12345) == 5 | (3 << 6)
    import ctypes
    c = mvx.coll()
    assert c.mvx_comm_set_phase_timing(12345, 1) == 5 | (3 << 6)
    assert c.mvx_comm_phase_times(12345, (ctypes.c_float * 4)()) == 5 | (3 << 6)


def test_plan_rejects_bad_arguments(mvx):
    with pytest.raises(ValueError):
        mvx.plan(mvx.COLL_ALLREDUCE, 0, 0, 10, 10, 102)
    with pytest.raises(ValueError):
        mvx.plan(mvx.COLL_ALLREDUCE, 4, 4, 10, 10, 102)
    with pytest.raises(ValueError):
        mvx.plan(mvx.COLL_REDUCE, 4, 0, 10, 10, 102, root=9)
    with pytest.raises(ValueError):
        mvx.plan(mvx.COLL_ALLREDUCE, 4, 0, 10, 99, 102)


def test_plan_phase_ranges_are_consistent(mvx):
    """Every send has a matching receive (same range) on the peer, and the
    data each rank combines is exactly what it receives."""
    for coll in (mvx.COLL_ALLREDUCE, mvx.COLL_REDUCE, mvx.COLL_REDUCE_SCATTER):
        for p in range(1, 9):
            for n in (3, 1000, 100000):
                for op, dt in ((102, 10), (100, 10)):
                    cn = [n + r for r in range(p)] if coll == mvx.COLL_REDUCE_SCATTER else None
                    P = [mvx.plan(coll, p, r, n, dt, op, p - 1, cn) for r in range(p)]
                    for r in range(p):
                        for s in range(p):
                            assert (P[r].a_send[s].off, P[r].a_send[s].cnt) == (P[s].a_recv[r].off, P[s].a_recv[r].cnt)
                            assert P[r].b_send[s].cnt == P[s].b_recv[r].cnt
                            if P[r].b_send[s].cnt:
                                assert P[r].b_send[s].off == P[s].b_recv[r].off
                            if P[r].a_recv[s].cnt:
                                assert (P[r].a_recv[s].off, P[r].a_recv[s].cnt) == (P[r].c_src_off, P[r].c_cnt)


def test_transport_table_is_read_only_as_far_as_the_caller_says(mvx):
    """mvx_comm_init_transport_ex reads `bytes` of the table: below the base
    (ctx + the four phase callbacks) it is an argument error, whatever the
    rest holds; a table with no callbacks is refused before any device call."""
    tp = __import__("importlib").import_module("mvapich-cce_amd.transport")
    h = ctypes.c_int()
    t = tp.Transport()
    L = mvx.coll()
    base = ctypes.sizeof(t) - 2 * ctypes.sizeof(ctypes.c_void_p)
    assert L.mvx_comm_init_transport_ex(ctypes.byref(h), 0, 2, 0, ctypes.byref(t), base - 1) == mvx.MPI_ERR_ARG
    assert L.mvx_comm_init_transport_ex(ctypes.byref(h), 0, 2, 0, ctypes.byref(t), ctypes.sizeof(t)) == mvx.MPI_ERR_ARG
    assert L.mvx_comm_init_transport(ctypes.byref(h), 0, 2, 0, ctypes.byref(t)) == mvx.MPI_ERR_ARG


def test_comm_knob_entry_points_reject_null_communicators(mvx):
    L = mvx.coll()
    code = 197                    # MPI_ERR_COMM | 3 << 6, as the reference's null-comm test
    st, err = ctypes.c_int(), ctypes.c_int()
    assert L.mvx_comm_set_graphs(12345, 1) == code
    assert L.mvx_comm_last_graph(12345, ctypes.byref(st), ctypes.byref(err)) == code
    assert L.mvx_comm_set_host_pipeline(12345, 1) == code
    assert L.mvx_comm_rccl_info(12345, None, None, None) == code
    assert L.mvx_comm_reap() == 0            # nothing parked in this process
    assert L.mvx_host_unregister(ctypes.c_void_p(4096)) != 0
