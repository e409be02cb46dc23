"""mvapich-cce_amd -- MI355X-native MPI reduction path (Python host mirror).

The product is in-tree shared libraries built from ``csrc/``:

* ``libmvx_hip.so`` -- hand-written HIP kernels for gfx950 behind the C-ABI of
  ``include/mvx_hip.h`` (``mvx_op_apply``, ``mvx_op_combine``, ...);
* ``libmvx.so`` -- the C host library of ``include/mvx_coll.h``:
  ``MPI_Reduce`` / ``MPI_Allreduce`` / ``MPI_Reduce_scatter`` /
  ``MPI_Op_create`` / ``MPI_Op_free`` / ``MPIR_SUM`` ... with the reference's
  handles and error codes, plans in the reference's combine order, RCCL for
  the data movement;
* ``libmvx_embed.so`` -- the same host library exporting only ``mvx_*``
  names (``include/mvx_embed.h``), for linking into MVAPICH itself
  (``integration/intra_mvx.c``).

This module binds them with ctypes and mirrors the reference's C interface
(same function names, argument meaning and return codes) so tests read like
the reference's ``examples/test/coll/*.c``.  It never computes anything
itself: if the libraries are missing it raises.
"""
import ctypes
import os

from . import consts as C  # noqa: F401  (re-exported handles)
from .consts import *  # noqa: F401,F403

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_HIP = os.path.join(HERE, "libmvx_hip.so")
LIB_COLL = os.path.join(HERE, "libmvx.so")

_hip = None
_coll = None


class NativeMissing(RuntimeError):
    pass


def build(verbose=False):
    """Compile both libraries in-tree (hipcc for gfx950, gcc for the host)."""
    import subprocess
    jobs = os.environ.get("MAX_JOBS", "4")
    cmd = ["make", "-C", os.path.join(HERE, "csrc"), "-j", jobs]
    if not verbose:
        cmd.insert(1, "-s")
    subprocess.check_call(cmd)


class Range(ctypes.Structure):
    _fields_ = [("off", ctypes.c_long), ("cnt", ctypes.c_long)]


MAXP = 64
MAXK = 64


class Plan(ctypes.Structure):
    """Mirror of ``mvx_plan`` (include/mvx_coll.h)."""
    _fields_ = [
        ("coll", ctypes.c_int), ("alg", ctypes.c_int), ("p", ctypes.c_int), ("rank", ctypes.c_int),
        ("root", ctypes.c_int), ("op", ctypes.c_int), ("dtype", ctypes.c_int), ("esize", ctypes.c_int),
        ("symmetric", ctypes.c_int), ("calls_uop", ctypes.c_int), ("count", ctypes.c_long),
        ("a_send", Range * MAXP), ("a_recv", Range * MAXP),
        ("has_combine", ctypes.c_int), ("k", ctypes.c_int), ("shape", ctypes.c_int), ("c_dst_tmp", ctypes.c_int),
        ("seg_heads", ctypes.c_ulonglong),
        ("leaf", ctypes.c_int * MAXK), ("leaf_fold", ctypes.c_int * MAXK),
        ("c_src_off", ctypes.c_long), ("c_cnt", ctypes.c_long), ("c_dst_off", ctypes.c_long),
        ("b_send", Range * MAXP), ("b_recv", Range * MAXP),
        ("opkind", ctypes.c_int), ("tree_swap", ctypes.c_int), ("chain_swap", ctypes.c_ulonglong),
        ("packed", ctypes.c_int),
    ]

    def masks(self):
        """(tree_mask, chain_mask) of a <= 8-leaf program (mvx_plan_masks)."""
        t, c = ctypes.c_uint(), ctypes.c_uint()
        rc = coll().mvx_plan_masks(ctypes.byref(self), ctypes.byref(t), ctypes.byref(c))
        if rc:
            raise ValueError("mvx_plan_masks rc=%d" % rc)
        return t.value, c.value

    def segments(self):
        """[(start, end)] of the program's tree segments."""
        heads = [q for q in range(self.k) if self.seg_heads >> q & 1] + [self.k]
        return list(zip(heads[:-1], heads[1:]))


class Tuning(ctypes.Structure):
    """Mirror of ``mvx_tuning`` (include/mvx_coll.h): device flavour + knobs."""
    _fields_ = [
        ("smp", ctypes.c_int), ("enable_shmem_collectives", ctypes.c_int), ("shmem_coll_ok", ctypes.c_int),
        ("disable_shmem_reduce", ctypes.c_int), ("disable_shmem_allreduce", ctypes.c_int),
        ("shmem_coll_reduce_threshold", ctypes.c_int), ("shmem_coll_allreduce_threshold", ctypes.c_int),
    ]


def _load():
    global _hip, _coll
    if _coll is not None:
        return
    if not (os.path.exists(LIB_HIP) and os.path.exists(LIB_COLL)):
        raise NativeMissing("libmvx_hip.so / libmvx.so not built: run __graft_entry__.build() "
                            "(there is no non-native fallback)")
    # If torch is in use it must own the HIP runtime: load it first so the
    # libamdhip64.so.7 / librccl.so.1 SONAMEs resolve to its copies.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    _hip = ctypes.CDLL(LIB_HIP, mode=ctypes.RTLD_GLOBAL)
    _coll = ctypes.CDLL(LIB_COLL, mode=ctypes.RTLD_GLOBAL)
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    pi = ctypes.POINTER(ctypes.c_int)
    pvp = ctypes.POINTER(ctypes.c_void_p)
    _hip.mvx_op_supported.argtypes = [i, i]
    _hip.mvx_dtype_extent.argtypes = [i]
    _hip.mvx_op_apply.argtypes = [i, i, vp, vp, sz, vp]
    _hip.mvx_op_combine.argtypes = [i, i, pvp, pvp, i, i, vp, sz, vp]
    _hip.mvx_op_program.argtypes = [i, i, pvp, pvp, i, ctypes.c_uint, ctypes.c_uint, vp, sz, vp]
    _hip.mvx_tree_mask.argtypes = [i]
    _hip.mvx_tree_mask.restype = ctypes.c_uint
    _hip.mvx_chain_mask.argtypes = [i]
    _hip.mvx_chain_mask.restype = ctypes.c_uint
    _hip.mvx_hip_set_launch.argtypes = [i, i]
    _hip.mvx_hip_set_launch.restype = None
    _hip.mvx_hip_last_kernel.restype = ctypes.c_char_p
    _hip.mvx_hip_last_kernel_symbol.restype = ctypes.c_char_p
    _hip.mvx_hip_last_launch.argtypes = [ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_int)]
    _hip.mvx_hip_last_launch.restype = None
    _hip.mvx_set_fortran_logical.argtypes = [i, i]
    c = _coll
    c.mvx_get_unique_id.argtypes = [vp]
    c.mvx_comm_init.argtypes = [pi, i, i, i, vp]
    c.mvx_comm_init_local.argtypes = [pi, i, i]
    c.mvx_comm_init_transport.argtypes = [pi, i, i, i, vp]
    c.mvx_comm_init_transport_ex.argtypes = [pi, i, i, i, vp, sz]
    c.mvx_comm_set_host_pipeline.argtypes = [i, i]
    c.mvx_comm_set_graphs.argtypes = [i, i]
    c.mvx_comm_last_graph.argtypes = [i, pi, pi]
    c.mvx_comm_graph_stats.argtypes = [i, pi, pi, ctypes.POINTER(ctypes.c_long)]
    c.mvx_comm_set_call_kinds.argtypes = [i, i]
    c.mvx_comm_reap.argtypes = []
    c.mvx_host_register_enable.argtypes = [i, sz]
    c.mvx_host_unregister.argtypes = [vp]
    c.mvx_host_invalidate.argtypes = [vp, sz]
    c.mvx_host_register.argtypes = [vp, sz]
    c.mvx_host_hooks_active.argtypes = []
    c.mvx_host_register_invalidations.restype = ctypes.c_long
    c.mvx_host_register_stats.argtypes = [ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_size_t),
                                          ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long)]
    c.mvx_host_register_deferred.argtypes = [ctypes.POINTER(ctypes.c_long)] * 4
    c.mvx_copy.argtypes = [vp, vp, sz]
    c.mvx_stream_synchronize.argtypes = [vp]
    c.mvx_comm_free.argtypes = [pi]
    c.mvx_comm_abort.argtypes = [pi]
    c.mvx_comm_rccl_native.argtypes = [i, i, vp, vp, sz, i, vp]
    c.mvx_comm_rccl_info.argtypes = [i, pi, pi, pi]
    c.mvx_comm_set_stream.argtypes = [i, vp]
    c.mvx_comm_reserve.argtypes = [i, sz]
    c.mvx_comm_set_exchange.argtypes = [i, i, i]
    c.mvx_comm_get_exchange.argtypes = [i, pi, pi]
    c.mvx_comm_last_exchange.argtypes = [i, pi]
    c.mvx_comm_set_phase_timing.argtypes = [i, i]
    c.mvx_comm_phase_times.argtypes = [i, ctypes.POINTER(ctypes.c_float)]
    c.MPI_Comm_size.argtypes = [i, pi]
    c.MPI_Comm_rank.argtypes = [i, pi]
    c.mvx_buffer_is_device.argtypes = [vp]
    for name in ("MPI_Allreduce", "PMPI_Allreduce", "mvx_coll_allreduce"):
        getattr(c, name).argtypes = [vp, vp, i, i, i, i]
    for name in ("MPI_Reduce", "PMPI_Reduce", "mvx_coll_reduce"):
        getattr(c, name).argtypes = [vp, vp, i, i, i, i, i]
    for name in ("MPI_Scan", "PMPI_Scan", "mvx_coll_scan"):
        getattr(c, name).argtypes = [vp, vp, i, i, i, i]
    c.mvx_scan_async.argtypes = [vp, vp, i, i, i, i, vp]
    c.mvx_scan_multi.argtypes = [pvp, pvp, i, i, i, i, pi, vp]
    for name in ("MPI_Reduce_scatter", "PMPI_Reduce_scatter", "mvx_coll_reduce_scatter"):
        getattr(c, name).argtypes = [vp, vp, pi, i, i, i]
    c.MPI_Op_create.argtypes = [vp, i, pi]
    c.mvx_op_create_device.argtypes = [vp, i, pi]
    c.MPI_Op_free.argtypes = [pi]
    c.MPI_Error_class.argtypes = [i, pi]
    c.mvx_allreduce_async.argtypes = [vp, vp, i, i, i, i, vp]
    c.mvx_reduce_async.argtypes = [vp, vp, i, i, i, i, i, vp]
    c.mvx_reduce_scatter_async.argtypes = [vp, vp, pi, i, i, i, vp]
    c.mvx_allreduce_multi.argtypes = [pvp, pvp, i, i, i, i, pi, vp]
    c.mvx_reduce_multi.argtypes = [pvp, pvp, i, i, i, i, i, pi, vp]
    c.mvx_reduce_scatter_multi.argtypes = [pvp, pvp, pi, i, i, i, pi, vp]
    c.mvx_plan_build.argtypes = [ctypes.POINTER(Plan), i, i, i, ctypes.c_long, pi, i, i, i]
    c.mvx_plan_masks.argtypes = [ctypes.POINTER(Plan), ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint)]
    c.mvx_plan_algorithm.argtypes = [i, i, ctypes.c_long, i]
    c.mvx_plan_build_kind.argtypes = [ctypes.POINTER(Plan), i, i, i, ctypes.c_long, pi, i, i, i, i]
    c.mvx_plan_algorithm_kind.argtypes = [i, i, ctypes.c_long, i, i]
    c.mvx_dtype_info.argtypes = [i, pi, pi]
    pt = ctypes.POINTER(Tuning)
    c.mvx_plan_build_tuned.argtypes = [ctypes.POINTER(Plan), i, i, i, ctypes.c_long, pi, i, i, i, i, pt]
    c.mvx_plan_algorithm_tuned.argtypes = [i, i, ctypes.c_long, i, i, pt]
    c.mvx_tuning_from_env.argtypes = [pt, i]
    pl = ctypes.POINTER(ctypes.c_long)
    _hip.mvx_type_contiguous.argtypes = [i, i, pi]
    _hip.mvx_type_free.argtypes = [pi]
    _hip.mvx_type_describe.argtypes = [i, pi, pi, pl, pl]
    c.MPI_Type_contiguous.argtypes = [i, i, pi]
    c.MPI_Type_vector.argtypes = [i, i, i, i, pi]
    c.MPI_Type_hvector.argtypes = [i, i, ctypes.c_long, i, pi]
    c.MPI_Type_indexed.argtypes = [i, pi, pi, i, pi]
    c.MPI_Type_hindexed.argtypes = [i, pi, pl, i, pi]
    c.MPI_Type_struct.argtypes = [i, pi, pl, pi, pi]
    c.MPI_Type_lb.argtypes = [i, pl]
    c.MPI_Type_ub.argtypes = [i, pl]
    _hip.mvx_type_layout.argtypes = [i, pi, pi, pl, pl, pl, pl]
    _hip.mvx_type_pack.argtypes = [i, vp, vp, sz, vp]
    _hip.mvx_type_unpack.argtypes = [i, vp, vp, sz, vp]
    _hip.mvx_op_element_size.argtypes = [i, i]
    c.MPI_Type_commit.argtypes = [pi]
    c.mvx_type_set_handle.argtypes = [i, i]
    c.MPI_Type_free.argtypes = [pi]
    c.MPI_Type_extent.argtypes = [i, pl]
    c.MPI_Type_size.argtypes = [i, pi]
    c.mvx_comm_get_tuning.argtypes = [i, pt]
    c.mvx_comm_set_tuning.argtypes = [i, pt]
    for name in ("MPIR_MAXF", "MPIR_MINF", "MPIR_SUM", "MPIR_PROD", "MPIR_LAND", "MPIR_BAND", "MPIR_LOR",
                 "MPIR_BOR", "MPIR_LXOR", "MPIR_BXOR", "MPIR_MAXLOC", "MPIR_MINLOC"):
        fn = getattr(c, name)
        fn.argtypes = [vp, vp, pi, pi]
        fn.restype = None


def hip():
    _load()
    return _hip


def coll():
    _load()
    return _coll


def loaded_paths():
    """Absolute paths of the native libraries this process has loaded."""
    _load()
    return [LIB_HIP, LIB_COLL]


# ---------------------------------------------------------------- plans ----

def plan(coll_kind, p, rank, count, dtype, op, root=0, recvcnts=None, opkind=None, tuning=None):
    """Rank `rank`'s plan; opkind (OPKIND_*) for a user op, None = predefined;
    tuning (a Tuning) for the device flavour, None = ch_shmem."""
    P = Plan()
    rc_arr = None
    if recvcnts is not None:
        rc_arr = (ctypes.c_int * p)(*recvcnts)
    if tuning is not None:
        rc = coll().mvx_plan_build_tuned(ctypes.byref(P), coll_kind, p, rank, count, rc_arr, dtype, op, root,
                                         opkind or 0, ctypes.byref(tuning))
    elif opkind is None:
        rc = coll().mvx_plan_build(ctypes.byref(P), coll_kind, p, rank, count, rc_arr, dtype, op, root)
    else:
        rc = coll().mvx_plan_build_kind(ctypes.byref(P), coll_kind, p, rank, count, rc_arr, dtype, op, root,
                                        opkind)
    if rc:
        raise ValueError("mvx_plan_build rc=%d" % rc)
    return P


def algorithm(coll_kind, p, total, dtype, opkind=None, tuning=None):
    if tuning is not None:
        return coll().mvx_plan_algorithm_tuned(coll_kind, p, total, dtype, opkind or 0, ctypes.byref(tuning))
    if opkind is None:
        return coll().mvx_plan_algorithm(coll_kind, p, total, dtype)
    return coll().mvx_plan_algorithm_kind(coll_kind, p, total, dtype, opkind)


def tuning_from_env(smp=True):
    """mvx_tuning_from_env: the knobs of an _SMP_ (smp) or ch_shmem build
    after the VIADEV_* environment.  Raises if the reference would exit."""
    t = Tuning()
    rc = coll().mvx_tuning_from_env(ctypes.byref(t), int(bool(smp)))
    if rc:
        raise ValueError("mvx_tuning_from_env rc=%d" % rc)
    return t


def smp_tuning(**knobs):
    """An _SMP_-flavour Tuning with the reference defaults, fields overridden
    by keyword (e.g. shmem_coll_allreduce_threshold=4096)."""
    t = Tuning(1, 1, 1, 0, 0, 1 << 10, 1 << 15)
    for k, v in knobs.items():
        setattr(t, k, v)
    return t


def dtype_info(dtype):
    e, s = ctypes.c_int(), ctypes.c_int()
    rc = coll().mvx_dtype_info(dtype, ctypes.byref(e), ctypes.byref(s))
    if rc:
        raise ValueError("unregistered datatype %d" % dtype)
    return e.value, s.value


def error_class(code):
    c = ctypes.c_int()
    coll().MPI_Error_class(code, ctypes.byref(c))
    return c.value


from .api import *  # noqa: E402,F401,F403
