"""The MVAPICH collops shim (integration/intra_mvx.c) on the CPU.

Compiled against the compile-check headers (integration/check/) with the
one-process runtime stand-in (integration/check/harness.c) and linked to
libmvx_embed.so.  Checks, without a GPU:
  * every struct field and runtime function the shim uses exists, spelled the
    same, in the reference's own headers (mpid/ch2/comm.h, ch_gen2/comm.h,
    datatype.h, mpiops.h, mpicoll.h, mpi.h) -- when /root/reference is here;
  * datatype translation: reference-shaped node trees (what type_contig.c,
    type_hvec.c, type_hind.c, type_struct.c store, bounds from the oracle's
    restatement) become libmvx types with the same lb / ub / extent / size,
    permanent types pass by handle, a node whose bounds disagree is refused;
  * op translation: predefined ops pass by handle, a user op is registered
    once per (handle, function, commute);
  * host buffers take MVAPICH's own path (the stand-in counts the calls);
  * the route is agreed across ranks (2-3 processes, the harness's board
    world): host buffers everywhere run MVAPICH's path on every rank after one
    route agreement per call (none for an empty call or under
    MVX_SHIM_ROUTE=local); a rank that wants libmvx takes every rank there,
    and a twin that cannot be created (no GPU here) fails the call on every
    rank alike, promptly, and stays failed.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(ROOT, "integration", "check")
SHIM = os.path.join(ROOT, "integration", "intra_mvx.c")
REF = "/root/reference"

INT, FLOAT, DOUBLE, UNSIGNED = 6, 10, 11, 7
FLOAT_INT, LB, UB = 17, 15, 16
MPI_SUM, MPI_MAXLOC, MPI_ERR_TYPE = 102, 111, 3


def _lib(smp=False, init=True):
    subprocess.check_call(["make", "-s", "-C", CHECK])
    # the package loads torch (if present) before libmvx*, so one HIP runtime
    # serves both: loaded first, the check library's libamdhip64.so.7 would
    # leave torch a second runtime that knows none of our pointers
    import importlib
    importlib.import_module("mvapich-cce_amd").coll()
    so = os.path.join(CHECK, "libintra_mvx_check_smp.so" if smp else "libintra_mvx_check.so")
    lib = ctypes.CDLL(so)
    vp, lg, i = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
    lib.h_basic.restype = vp
    lib.h_basic.argtypes = [i, lg, lg, lg, lg]
    lib.h_contig.restype = vp
    lib.h_contig.argtypes = [i, vp, lg, lg, lg, lg]
    lib.h_hvector.restype = vp
    lib.h_hvector.argtypes = [i, i, lg, vp, lg, lg, lg, lg]
    lib.h_hindexed.restype = vp
    lib.h_hindexed.argtypes = [i, vp, vp, vp, lg, lg, lg, lg]
    lib.h_struct.restype = vp
    lib.h_struct.argtypes = [i, vp, vp, vp, lg, lg, lg, lg]
    lib.h_self.argtypes = [vp]
    lib.h_translate.argtypes = [vp, ctypes.POINTER(i)]
    lib.h_op_translate.argtypes = [i, ctypes.POINTER(i)]
    lib.h_allreduce.argtypes = [vp, vp, i, vp, i]
    lib.h_reduce.argtypes = [vp, vp, i, vp, i, i]
    lib.h_reduce_scatter.argtypes = [vp, vp, vp, vp, i]
    lib.h_scan.argtypes = [vp, vp, i, vp, i]
    if init:
        assert lib.h_init() == 0
    return lib


@pytest.fixture(scope="module")
def shim(mvx):
    return _lib()


class Nodes:
    """Builds each type twice: in the oracle (the reference's bounds rules)
    and as the node tree the reference's constructors would have stored."""

    def __init__(self, lib, O):
        self.lib, self.O = lib, O

    def _bounds(self, rc_h):
        rc, h = rc_h
        assert rc == 0
        rc, lb, ub, ext, size = self.O.type_bounds(h)
        assert rc == 0
        return h, (lb, ub, ext, size)

    def basic(self, h):
        rc, lb, ub, ext, size = self.O.type_bounds(h)
        assert rc == 0
        return h, self.lib.h_basic(h, lb, ub, ext, size)

    def contig(self, count, old):
        oh, on = old
        h, b = self._bounds(self.O.type_contiguous(count, oh))
        return h, self.lib.h_contig(count, on, *b)

    def vector(self, count, bl, stride, old):
        """type_vec.c:71-83: contiguous when blocklen == stride or count == 1,
        else an hvector with the stride in bytes"""
        oh, on = old
        h, b = self._bounds(self.O.type_vector(count, bl, stride, oh))
        if bl == stride or count == 1:
            return h, self.lib.h_contig(count * bl, on, *b)
        ext = self.O.type_bounds(oh)[3]
        return h, self.lib.h_hvector(count, bl, stride * ext, on, *b)

    def hvector(self, count, bl, stride, old):
        oh, on = old
        h, b = self._bounds(self.O.type_hvector(count, bl, stride, oh))
        return h, self.lib.h_hvector(count, bl, stride, on, *b)

    def indexed(self, bls, idx, old):
        """type_ind.c:103-126: a null type for zero total blocklen, else an
        hindexed with byte displacements"""
        oh, on = old
        h, b = self._bounds(self.O.type_indexed(len(bls), bls, idx, oh))
        if sum(bls) == 0:
            return h, self.lib.h_contig(0, self.basic(INT)[1], *b)
        ext = self.O.type_bounds(oh)[3]
        return h, self._hind(bls, [x * ext for x in idx], on, b)

    def _hind(self, bls, idx, on, b):
        cb = (ctypes.c_int * len(bls))(*bls)
        ci = (ctypes.c_long * len(idx))(*idx)
        return self.lib.h_hindexed(len(bls), cb, ci, on, *b)

    def struct(self, bls, idx, olds):
        h, b = self._bounds(self.O.type_struct(len(bls), bls, idx, [o[0] for o in olds]))
        cb = (ctypes.c_int * len(bls))(*bls)
        ci = (ctypes.c_long * len(idx))(*idx)
        co = (ctypes.c_void_p * len(olds))(*[o[1] for o in olds])
        return h, self.lib.h_struct(len(bls), cb, ci, co, *b)


def _cases(N):
    i, f, d = N.basic(INT), N.basic(FLOAT), N.basic(DOUBLE)
    lb, ub = N.basic(LB), N.basic(UB)
    vec = N.vector(4, 2, 3, i)
    return {
        "contig3f": N.contig(3, f),
        "vec_hv": vec,
        "vec_as_contig": N.vector(3, 2, 2, d),
        "indexed": N.indexed([1, 2, 1], [0, 3, 7], d),
        "indexed_null": N.indexed([0, 0], [1, 4], i),
        "hvec_neg": N.hvector(3, 1, -16, i),
        "struct_id_ub": N.struct([1, 1, 1], [0, 8, 24], [i, d, ub]),
        "struct_lb": N.struct([1, 1, 1, 1], [-8, 0, 4, 16], [lb, i, f, ub]),
        "contig_of_vec": N.contig(2, vec),
        "nest": N.struct([1, 2], [0, 16], [N.contig(2, i), N.hvector(2, 1, 24, d)]),
        "float_int": N.basic(FLOAT_INT),
    }


def test_fields_exist_in_reference_headers():
    """Every `->field` the shim reads and every MPIR_ / MPI_ runtime name it
    calls is spelled as in the reference's headers (the compile-check
    headers could otherwise drift from the real ones)."""
    if not os.path.isdir(REF):
        pytest.skip("reference tree not present")
    src = open(SHIM).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    # accesses through the reference's objects (d: MPIR_DATATYPE, comm /
    # leaders: MPIR_COMMUNICATOR, o: MPIR_OP, the collops tables)
    fields = set(re.findall(r"\b(?:d|comm|leaders|o|MPIR_COMM_WORLD|MPIR_intra_collops)\s*->\s*([A-Za-z_]\w*)", src))
    fields |= set(re.findall(r"\btable\.([A-Za-z_]\w*)", src))
    assert {"np", "local_rank", "self", "dte_type", "old_types", "Bcast", "ref_count"} <= fields
    heads = ["mpid/ch2/comm.h", "mpid/ch_gen2/comm.h", "mpid/ch2/datatype.h", "include/mpiops.h",
             "include/mpicoll.h"]
    text = "\n".join(open(os.path.join(REF, h), errors="replace").read() for h in heads)
    decl = set(re.findall(r"[\s*]([A-Za-z_]\w*)\s*(?:\[[^\]]*\])?\s*[;,)]", text))
    decl |= set(re.findall(r"\(\s*\*\s*([A-Za-z_]\w*)\s*\)", text))     # collops members
    missing = sorted(fields - decl)
    assert not missing, missing
    calls = set(re.findall(r"\b(MPI_\w+|MPIR_\w+)\b", src)) - {"MPIR_mvx_collops", "MPIR_mvx_collops_init"}
    defs = "\n".join(open(os.path.join(REF, h), errors="replace").read()
                     for h in ["include/mpi.h", "include/mpiimpl.h", "include/mpicoll.h",
                               "mpid/ch2/datatype.h", "mpid/ch2/comm.h", "include/mpi_errno.h",
                               "include/mpi_error.h", "src/fortran/include/mpi_fort.h"])
    missing = sorted(c for c in calls if not re.search(r"\b%s\b" % c, defs))
    assert not missing, missing
    # the nodetype names the shim switches on
    for k in ("MPIR_CONTIG", "MPIR_HVECTOR", "MPIR_HINDEXED", "MPIR_STRUCT"):
        assert k in text


def test_type_translation_matches_reference_bounds(mvx, oracle, shim):
    N = Nodes(shim, oracle)
    for name, (oh, node) in _cases(N).items():
        t = ctypes.c_int()
        rc = shim.h_translate(node, ctypes.byref(t))
        assert rc == 0, name
        if name == "float_int":
            assert t.value == FLOAT_INT
            continue
        _, lb, ub, ext, size = oracle.type_bounds(oh)
        lay = mvx.type_layout(t.value)
        assert (lay["lb"], lay["ub"]) == (lb, ub), name
        assert mvx.MPI_Type_extent(t.value)[1] == ext, name
        assert mvx.MPI_Type_size(t.value)[1] == size, name
        # cached: the same node translates to the same libmvx type
        t2 = ctypes.c_int()
        assert shim.h_translate(node, ctypes.byref(t2)) == 0 and t2.value == t.value


def test_mismatched_bounds_are_refused(mvx, oracle, shim):
    N = Nodes(shim, oracle)
    f = N.basic(FLOAT)
    rc, lb, ub, ext, size = oracle.type_bounds(oracle.type_contiguous(3, FLOAT)[1])
    bad = shim.h_contig(3, f[1], lb, ub + 4, ext + 4, size)
    t = ctypes.c_int()
    assert shim.h_translate(bad, ctypes.byref(t)) == MPI_ERR_TYPE


def test_op_translation(shim):
    o = ctypes.c_int()
    for op in range(100, 112):
        assert shim.h_op_translate(op, ctypes.byref(o)) == 0 and o.value == op
    u1 = shim.h_op_create(1)
    u2 = shim.h_op_create(0)
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert shim.h_op_translate(u1, ctypes.byref(a)) == 0
    assert shim.h_op_translate(u1, ctypes.byref(b)) == 0 and a.value == b.value
    assert shim.h_op_translate(u2, ctypes.byref(c)) == 0 and c.value != a.value
    assert a.value >= 200 and c.value >= 200     # libmvx user-op handles


def test_host_buffers_take_mvapich_path(mvx, oracle, shim, monkeypatch):
    monkeypatch.delenv("MVX_HOST_BUFFERS", raising=False)
    N = Nodes(shim, oracle)
    f = N.basic(FLOAT)
    s = np.arange(30, dtype=np.float32)
    r = np.zeros(30, np.float32)
    before = shim.h_host_calls()
    assert shim.h_allreduce(s.ctypes.data, r.ctypes.data, 30, f[1], MPI_SUM) == 0
    assert shim.h_reduce(s.ctypes.data, r.ctypes.data, 30, f[1], MPI_SUM, 0) == 0
    cn = (ctypes.c_int * 1)(30)
    assert shim.h_reduce_scatter(s.ctypes.data, r.ctypes.data, cn, f[1], MPI_SUM) == 0
    assert shim.h_scan(s.ctypes.data, r.ctypes.data, 30, f[1], MPI_SUM) == 0
    assert shim.h_host_calls() == before + 4
    assert np.array_equal(r, s)


def test_smp_build_loads(mvx):
    lib = _lib(smp=True)
    assert lib.h_host_calls() == 0


def test_check_headers_match_reference_layout():
    """The compile-check headers lay out every member the shim reads at the
    offsets the reference's own headers give (plain ch_shmem and the _SMP_
    devices' ch_gen2 communicator), and the committed ref_layout.h -- which
    layout_assert.c holds the check build to with _Static_assert -- is what
    those headers give today (integration/check/ref_layout.py)."""
    if not os.path.isdir(REF):
        pytest.skip("reference tree not present")
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "ref_layout", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "integration", "check", "ref_layout.py"))
    rl = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rl)
    lay = rl.reference_layouts(REF)
    assert rl.check_layouts(False) == lay["plain"]
    assert rl.check_layouts(True) == lay["smp"]
    names = dict(lay["smp"])
    # the _SMP_ communicator carries ch_gen2's mutex pointer and RDMA
    # collective members before the shmem fields the shim reads
    assert int(names["comm_t.collops"]) > int(dict(lay["plain"])["comm_t.collops"])
    with open(os.path.join(os.path.dirname(rl.__file__), "ref_layout.h")) as f:
        assert f.read() == rl.header_text(lay)


def _world(np_, scenario, envs=None, timeout=120):
    """np_ shim_worker.py processes sharing one harness board; their reports"""
    import json
    import sys
    import tempfile
    d = tempfile.mkdtemp(prefix="mvx_shim_")
    board = os.path.join(d, "board")
    with open(board, "wb") as f:
        f.write(b"\0" * 16384)
    procs = []
    for r in range(np_):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.pop("MVX_HOST_BUFFERS", None)
        env.pop("MVX_SHIM_ROUTE", None)
        env.update((envs or {}).get(r, {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "shim_worker.py"), str(r),
                                       str(np_), board, os.path.join(d, "r%d.json" % r), scenario], env=env))
    try:
        rcs = [p.wait(timeout=timeout) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert rcs == [0] * np_, rcs
    reps = []
    for r in range(np_):
        with open(os.path.join(d, "r%d.json" % r)) as f:
            reps.append(json.load(f))
    return reps


@pytest.mark.parametrize("np_", [2, 3])
def test_route_agreed_host_buffers_everywhere(mvx, np_):
    """Host buffers on every rank: every call runs MVAPICH's own function on
    every rank, after exactly one route agreement; an empty call and
    MVX_SHIM_ROUTE=local agree nothing."""
    for rep in _world(np_, "route"):
        calls = {c["name"]: c for c in rep["calls"]}
        for name in ("allreduce", "reduce", "reduce_scatter", "scan", "allreduce_again"):
            assert calls[name] == dict(calls[name], rc=0, agree=1, host=1), (rep["rank"], name, calls[name])
        assert calls["empty"]["agree"] == 0 and calls["empty"]["rc"] == 0
        assert calls["local"] == dict(calls["local"], rc=0, agree=0, host=1), calls["local"]


def test_route_one_rank_wanting_libmvx_takes_every_rank(mvx):
    """MVX_HOST_BUFFERS=1 on rank 0 only (the rank-local rule would send rank
    0 to libmvx and rank 1 to MVAPICH's path: a hang).  Agreed, every rank
    goes to libmvx; with no GPU here the twin cannot be created, so every
    rank fails the call (MPI_ERR_OTHER) without entering RCCL, within
    seconds, and every later call fails the same way with no second
    creation attempt (one route agreement per call, no creation
    agreements)."""
    reps = _world(2, "want", {0: {"MVX_HOST_BUFFERS": "1"}})
    for rep in reps:
        first, *rest = rep["calls"]
        assert first["rc"] == 15 and first["host"] == 0, rep
        # route + the creation agreement (device check / id) that stopped it
        assert first["agree"] == 2, first
        assert first["s"] < 30, first
        for c in rest:
            assert c["rc"] == 15 and c["host"] == 0 and c["agree"] == 1, c


@pytest.mark.parametrize("np_", [2, 3])
def test_route_kinds_count_only_the_buffers_a_rank_touches(mvx, np_):
    """Buffer kinds mixed within a rank (the harness treats chosen host
    arrays as device memory).  The route agreement's second int -- some rank
    touches host memory -- is 1 whenever any rank's touched buffers include
    host memory, whichever of its buffers it is: a device sendbuf beside a
    host recvbuf is host (round 5 reported it as device, and MVX_KINDS_DEVICE
    then failed that rank alone).  A non-root's Reduce recvbuf is never
    touched, so a host one there leaves the call all-device.  One route
    agreement per call (plus the twin's creation agreement at the first,
    which fails here: no GPU)."""
    root = np_ - 1
    for rep in _world(np_, "kinds_cpu"):
        r = rep["rank"]
        calls = {c["name"]: c for c in rep["calls"]}
        want = {"reduce_dh": (r == root, 1), "allreduce_dh": (1, 1), "rs_hd": (r == 0, 1),
                "reduce_dd": (0, 0), "allreduce_dd": (0, 0)}
        for name, (mine_host, all_host) in want.items():
            c = calls[name]
            assert c["route_mine"][0] == 1, (r, name, c)      # every rank touches a device buffer
            assert c["route_mine"][1] == int(mine_host), (r, name, c)
            assert c["route_all"] == [1, all_host, 0], (r, name, c)
            assert c["rc"] == 15 and c["host"] == 0, (r, name, c)
            assert c["agree"] == (2 if name == "reduce_dh" else 1), (r, name, c)


def test_translation_failure_on_one_rank_fails_every_rank(mvx):
    """Rank 1's datatype node does not rebuild to the reference's bounds.
    The shim translates before it agrees the route, so the agreement carries
    rank 1's MPI_ERR_TYPE: both ranks return it, promptly, after one
    agreement and without creating the twin (round 5 translated after the
    agreement: rank 1 failed alone while rank 0 entered the collective).
    The next call, with a good type everywhere, goes on to the twin."""
    reps = _world(2, "xlate", {0: {"MVX_HOST_BUFFERS": "1"}, 1: {"MVX_HOST_BUFFERS": "1"}})
    for rep in reps:
        bad, good = rep["calls"]
        assert bad["rc"] == MPI_ERR_TYPE and bad["agree"] == 1 and bad["host"] == 0, (rep["rank"], bad)
        assert bad["route_all"] == [1, 1, MPI_ERR_TYPE] and bad["s"] < 30, (rep["rank"], bad)
        assert bad["route_mine"][2] == (MPI_ERR_TYPE if rep["rank"] == 1 else 0), (rep["rank"], bad)
        assert good["rc"] == 15 and good["agree"] == 2 and good["route_all"] == [1, 1, 0], (rep["rank"], good)
