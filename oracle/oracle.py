"""TEST INFRASTRUCTURE: ctypes binding of oracle/liboracle.so.

The oracle is the CPU restatement of the reference reduction path
(oracle/cpu_ops.c restates src/coll/global_ops.c; oracle/coll_sim.c replays
the src/coll/intra_fns_new.c schedules).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import this module; the product package never
does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

ALG_NONE, ALG_RECDBL, ALG_RABENSEIFNER, ALG_BINOMIAL, ALG_RS_HALVING, ALG_RS_PAIRWISE = range(6)
ALG_RS_RECDBL = 7
COLL_ALLREDUCE, COLL_REDUCE, COLL_REDUCE_SCATTER = 1, 2, 3

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.orc_dtype_info.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.orc_op.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int]
        L.orc_set_flog.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_set_flog.restype = None
        L.orc_call.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int]
        L.orc_allreduce.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_reduce.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_reduce_scatter.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                         ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_int)]
        L.orc_scan.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_int,
                               ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_algorithm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int]
        L.orc_algorithm_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int]
        L.orc_user_op_set.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.orc_smp_set.argtypes = [ctypes.c_int] * 7
        L.orc_type_contiguous.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_type_free.argtypes = [ctypes.POINTER(ctypes.c_int)]
        pint, plong = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_long)
        L.orc_type_vector.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, pint]
        L.orc_type_hvector.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int, pint]
        L.orc_type_indexed.argtypes = [ctypes.c_int, pint, pint, ctypes.c_int, pint]
        L.orc_type_hindexed.argtypes = [ctypes.c_int, pint, plong, ctypes.c_int, pint]
        L.orc_type_struct.argtypes = [ctypes.c_int, pint, plong, pint, pint]
        L.orc_type_commit.argtypes = [ctypes.c_int]
        L.orc_type_bounds.argtypes = [ctypes.c_int, plong, plong, plong, plong]
        L.orc_type_copy.argtypes = [vp, vp, ctypes.c_long, ctypes.c_int]
        L.orc_threads_coll.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                       ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_threads_coll.restype = ctypes.c_double
        L.orc_fill.argtypes = [vp, ctypes.c_long, ctypes.c_int, ctypes.c_int]
        L.orc_fill.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def dtype_info(dtype):
    e, s = ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_dtype_info(dtype, ctypes.byref(e), ctypes.byref(s))
    if rc:
        raise ValueError("datatype %d not registered" % dtype)
    return e.value, s.value


def op(op_handle, dtype, invec, inoutvec, count):
    """inoutvec = invec op inoutvec (in place, numpy uint8 views). Returns rc.
    User op handles (user_op_set) call the registered function."""
    return lib().orc_call(op_handle, dtype, _ptr(invec), _ptr(inoutvec), count)


def set_fortran_logical(true_value, false_value):
    """MPIR_F_TRUE / MPIR_F_FALSE of MPI_LOGICAL (default 1 / 0)."""
    lib().orc_set_flog(true_value, false_value)


def _ptrs(bufs):
    arr = (ctypes.c_void_p * len(bufs))()
    for i, b in enumerate(bufs):
        arr[i] = b.ctypes.data
    return arr


def allreduce(sends, recvs, count, dtype, op_handle):
    p = len(sends)
    rc = (ctypes.c_int * p)()
    lib().orc_allreduce(p, _ptrs(sends), _ptrs(recvs), count, dtype, op_handle, rc)
    return list(rc)


def reduce(sends, recvs, count, dtype, op_handle, root):
    p = len(sends)
    rc = (ctypes.c_int * p)()
    lib().orc_reduce(p, _ptrs(sends), _ptrs(recvs), count, dtype, op_handle, root, rc)
    return list(rc)


def reduce_scatter(sends, recvs, recvcnts, dtype, op_handle):
    p = len(sends)
    rc = (ctypes.c_int * p)()
    cn = (ctypes.c_int * p)(*recvcnts)
    lib().orc_reduce_scatter(p, _ptrs(sends), _ptrs(recvs), cn, dtype, op_handle, rc)
    return list(rc)


def scan(sends, recvs, count, dtype, op_handle):
    p = len(sends)
    rc = (ctypes.c_int * p)()
    lib().orc_scan(p, _ptrs(sends), _ptrs(recvs), count, dtype, op_handle, rc)
    return list(rc)


def algorithm(coll, p, total_count, dtype, op=None):
    if op is None:
        return lib().orc_algorithm(coll, p, total_count, dtype)
    return lib().orc_algorithm_op(coll, p, total_count, dtype, op)


def user_op_set(handle, fn_addr, commute):
    """Register an MPI_User_function (C address) as user op `handle` (200..263)."""
    return lib().orc_user_op_set(handle, fn_addr, commute)


def threads_coll(coll, sends, recvs, tmps, count, dtype, op, root=0, recvcnts=None, reps=1):
    """The reference schedule on len(sends) host threads (CPU baseline);
    returns seconds per collective.  tmps[r] must hold 2 x total elements."""
    p = len(sends)
    cn = (ctypes.c_int * p)(*recvcnts) if recvcnts is not None else None
    return lib().orc_threads_coll(coll, p, _ptrs(sends), _ptrs(recvs), _ptrs(tmps), count, cn, dtype, op, root,
                                  reps)


def type_contiguous(count, oldtype):
    """MPI_Type_contiguous in the oracle's own table: (rc, handle)."""
    h = ctypes.c_int()
    rc = lib().orc_type_contiguous(count, oldtype, ctypes.byref(h))
    return rc, h.value


def _ia(vals, ct=ctypes.c_int):
    return (ct * max(len(vals), 1))(*vals)


def type_vector(count, blocklen, stride, oldtype):
    h = ctypes.c_int()
    rc = lib().orc_type_vector(count, blocklen, stride, oldtype, ctypes.byref(h))
    return rc, h.value


def type_hvector(count, blocklen, stride, oldtype):
    h = ctypes.c_int()
    rc = lib().orc_type_hvector(count, blocklen, stride, oldtype, ctypes.byref(h))
    return rc, h.value


def type_indexed(count, blocklens, indices, oldtype):
    h = ctypes.c_int()
    rc = lib().orc_type_indexed(count, _ia(blocklens), _ia(indices), oldtype, ctypes.byref(h))
    return rc, h.value


def type_hindexed(count, blocklens, indices, oldtype):
    h = ctypes.c_int()
    rc = lib().orc_type_hindexed(count, _ia(blocklens), _ia(indices, ctypes.c_long), oldtype, ctypes.byref(h))
    return rc, h.value


def type_struct(count, blocklens, indices, types):
    h = ctypes.c_int()
    rc = lib().orc_type_struct(count, _ia(blocklens), _ia(indices, ctypes.c_long), _ia(types), ctypes.byref(h))
    return rc, h.value


def type_commit(handle):
    return lib().orc_type_commit(handle)


def type_bounds(handle):
    """(rc, lb, ub, extent, size)"""
    v = [ctypes.c_long() for _ in range(4)]
    rc = lib().orc_type_bounds(handle, *[ctypes.byref(x) for x in v])
    return (rc,) + tuple(x.value for x in v)


def type_copy(dst, src, n, handle):
    """n elements, type-map bytes only (numpy buffers)."""
    return lib().orc_type_copy(_ptr(dst), _ptr(src), n, handle)


def type_free(handle):
    h = ctypes.c_int(handle)
    return lib().orc_type_free(ctypes.byref(h))


SMP_DEFAULTS = dict(enable=1, ok=1, dis_red=0, dis_ar=0, thr_red=1 << 10, thr_ar=1 << 15)


def smp_set(smp, **knobs):
    """Replay the _SMP_ builds' intra_shmem_* collops (smp=1) or the ch_shmem
    build's (smp=0).  knobs: enable, ok, dis_red, dis_ar, thr_red, thr_ar."""
    k = dict(SMP_DEFAULTS)
    k.update(knobs)
    return lib().orc_smp_set(int(smp), k["enable"], k["ok"], k["dis_red"], k["dis_ar"], k["thr_red"],
                             k["thr_ar"])


class smp_flavour:
    """Context manager: the oracle replays the _SMP_ collops inside."""

    def __init__(self, **knobs):
        self.knobs = knobs

    def __enter__(self):
        smp_set(1, **self.knobs)
        return self

    def __exit__(self, *exc):
        smp_set(0)
        return False


def fill(nbytes_or_array, n, dist, rank):
    a = nbytes_or_array
    lib().orc_fill(_ptr(a), n, dist, rank)
    return a
