"""Reference-shaped entry points over libmvx.so / libmvx_hip.so.

Buffers may be torch tensors (device or host), numpy arrays (host) or raw
integer addresses.  Return values are the C library's MPI error codes,
exactly as the reference's MPI_* functions return them.
"""
import ctypes

from . import coll, hip
from .consts import COLL_ALLREDUCE, COLL_REDUCE, COLL_REDUCE_SCATTER  # noqa: F401

__all__ = [
    "addr", "stream_handle", "op_apply", "op_combine", "op_program", "Comm",
    "MPI_Allreduce", "MPI_Reduce", "MPI_Reduce_scatter", "MPI_Scan", "MPI_Op_create", "MPI_Op_free", "op_create_device",
    "MPIR_call", "op_errno", "last_kernel", "last_kernel_symbol", "last_launch", "set_launch",
    "set_fortran_logical", "comm_reap", "host_register_enable", "host_unregister", "host_register_stats",
    "host_hooks_active", "host_invalidate", "host_register_deferred",
    "MPI_Type_contiguous", "MPI_Type_commit", "MPI_Type_free", "MPI_Type_extent", "MPI_Type_size",
    "MPI_Type_vector", "MPI_Type_hvector", "MPI_Type_indexed", "MPI_Type_hindexed", "MPI_Type_struct",
    "MPI_Type_lb", "MPI_Type_ub", "type_layout", "type_set_handle", "type_pack", "type_unpack",
]


def addr(buf):
    """Address of a tensor / ndarray / int (None -> 0)."""
    if buf is None:
        return 0
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):
        return buf.data_ptr()
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data
    raise TypeError("cannot take the address of %r" % type(buf))


def stream_handle(stream=None):
    """hipStream_t of a torch stream (default: torch's current stream)."""
    if isinstance(stream, int):
        return stream
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _pp(ptrs):
    arr = (ctypes.c_void_p * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = addr(p) or None
    return arr


def op_apply(op, dtype, invec, inoutvec, n, stream=None):
    """inoutvec = invec op inoutvec on the device (stream-ordered)."""
    return hip().mvx_op_apply(op, dtype, addr(invec), addr(inoutvec), n, stream_handle(stream))


def op_combine(op, dtype, srcs, dst, n, shape=0, folds=None, stream=None):
    """dst = shape-combine of leaves srcs (each optionally folded)."""
    k = len(srcs)
    fo = _pp(folds) if folds is not None else None
    return hip().mvx_op_combine(op, dtype, _pp(srcs), fo, k, shape, addr(dst), n, stream_handle(stream))


def op_program(op, dtype, srcs, dst, n, tree_mask, chain_mask, folds=None, stream=None):
    """dst = the combine program (tree steps, then chain) over leaves srcs."""
    fo = _pp(folds) if folds is not None else None
    return hip().mvx_op_program(op, dtype, _pp(srcs), fo, len(srcs), tree_mask, chain_mask, addr(dst), n,
                                stream_handle(stream))


def set_launch(block_cap=0, nt_min_log2=0):
    """Grid cap (blocks) and non-temporal threshold (log2 bytes, -1 = never)."""
    hip().mvx_hip_set_launch(block_cap, nt_min_log2)


def last_kernel():
    return hip().mvx_hip_last_kernel().decode()


def last_kernel_symbol():
    """The last launched kernel template, as rocprofv3 names it."""
    return hip().mvx_hip_last_kernel_symbol().decode()


def last_launch():
    """(grid blocks, dynamic LDS bytes, resident blocks per CU) of the last launch."""
    b, lds, occ = ctypes.c_uint(), ctypes.c_size_t(), ctypes.c_int()
    hip().mvx_hip_last_launch(ctypes.byref(b), ctypes.byref(lds), ctypes.byref(occ))
    return b.value, lds.value, occ.value


def set_fortran_logical(true_value, false_value):
    """MPI_LOGICAL's .TRUE. / .FALSE. words (mvx_set_fortran_logical; the
    reference's MPIR_F_TRUE / MPIR_F_FALSE), on the current device."""
    return hip().mvx_set_fortran_logical(true_value, false_value)


# ------------------------------------------------------------- communicators

class Comm:
    """An MPI_Comm handle of libmvx.so."""

    def __init__(self, handle, rank, size, local):
        self.handle, self.rank, self.size, self.local = handle, rank, size, local

    @classmethod
    def from_torch_distributed(cls, device=None):
        """One rank per GPU: RCCL communicator bootstrapped over the already
        initialised torch.distributed process group (any backend)."""
        import torch
        import torch.distributed as dist
        rank, size = dist.get_rank(), dist.get_world_size()
        if device is None:
            device = torch.cuda.current_device()
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            rc = coll().mvx_get_unique_id(uid)
            if rc:
                raise RuntimeError("mvx_get_unique_id rc=%d" % rc)
        box = [bytes(uid.raw) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = ctypes.create_string_buffer(box[0], 128)
        h = ctypes.c_int()
        rc = coll().mvx_comm_init(ctypes.byref(h), rank, size, device, uid)
        if rc:
            raise RuntimeError("mvx_comm_init rc=%d" % rc)
        return cls(h.value, rank, size, False)

    @classmethod
    def from_transport(cls, transport, device=None):
        """One rank per process with a host transport (mvx_comm_init_transport),
        e.g. transport.TorchP2PTransport over an initialised gloo group; several
        processes may share one GPU."""
        import torch
        import torch.distributed as dist
        rank, size = dist.get_rank(), dist.get_world_size()
        if device is None:
            device = torch.cuda.current_device()
        h = ctypes.c_int()
        t = transport.struct()
        rc = coll().mvx_comm_init_transport_ex(ctypes.byref(h), rank, size, device, ctypes.byref(t),
                                               ctypes.sizeof(t))
        if rc:
            raise RuntimeError("mvx_comm_init_transport rc=%d" % rc)
        c = cls(h.value, rank, size, False)
        c.transport = transport      # keeps the callbacks alive
        return c

    @classmethod
    def local_ranks(cls, size, device=0):
        """`size` virtual ranks on one device (use the *_multi methods)."""
        h = ctypes.c_int()
        rc = coll().mvx_comm_init_local(ctypes.byref(h), size, device)
        if rc:
            raise RuntimeError("mvx_comm_init_local rc=%d" % rc)
        return cls(h.value, 0, size, True)

    def free(self):
        h = ctypes.c_int(self.handle)
        coll().mvx_comm_free(ctypes.byref(h))

    def abort(self):
        """mvx_comm_abort: tear down without waiting for outstanding
        transfers (ncclCommAbort)."""
        h = ctypes.c_int(self.handle)
        return coll().mvx_comm_abort(ctypes.byref(h))

    def set_host_pipeline(self, on=True):
        """Host buffers at p > 1 through the sliced pipeline (every rank must
        then pass host buffers) instead of HBM mirrors (mvx_comm_set_host_pipeline)."""
        return coll().mvx_comm_set_host_pipeline(self.handle, 1 if on else 0)

    def set_graphs(self, on=True):
        """Capture device calls into HIP graphs and replay them (mvx_comm_set_graphs)."""
        return coll().mvx_comm_set_graphs(self.handle, 1 if on else 0)

    def set_call_kinds(self, kinds):
        """mvx_comm_set_call_kinds: every rank's buffer kinds in the next
        blocking call, agreed by the caller (KINDS_UNKNOWN / _DEVICE / _HOST)."""
        return coll().mvx_comm_set_call_kinds(self.handle, kinds)

    def graph_stats(self):
        """{live, retired, destroyed}: graphs held (replayable / kept but never
        replayed) and execs destroyed mid-life (mvx_comm_graph_stats)."""
        live, ret, dst = ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
        rc = coll().mvx_comm_graph_stats(self.handle, ctypes.byref(live), ctypes.byref(ret), ctypes.byref(dst))
        if rc:
            raise RuntimeError("mvx_comm_graph_stats rc=%d" % rc)
        return {"live": live.value, "retired": ret.value, "destroyed": dst.value}

    def last_graph(self):
        """(state, error) of the last call (mvx_comm_last_graph): state 0
        eager, 1 replayed, 2 captured and launched; error the failed
        capture's code that turned graphs off (0: none)."""
        st, err = ctypes.c_int(), ctypes.c_int()
        rc = coll().mvx_comm_last_graph(self.handle, ctypes.byref(st), ctypes.byref(err))
        if rc:
            raise RuntimeError("mvx_comm_last_graph rc=%d" % rc)
        return st.value, err.value

    def set_stream(self, stream=None):
        return coll().mvx_comm_set_stream(self.handle, stream_handle(stream))

    def rccl_native(self, coll_kind, sendbuf, recvbuf, count, dtype, stream=None):
        """Ablation only: RCCL's own ncclAllReduce / ncclReduceScatter
        (ncclSum) on this communicator (mvx_comm_rccl_native) -- not the
        reference's combine order; never a substitute for the MPI calls."""
        return coll().mvx_comm_rccl_native(self.handle, coll_kind, addr(sendbuf), addr(recvbuf), count, dtype,
                                           stream_handle(stream))

    def rccl_info(self):
        """RCCL's own view (mvx_comm_rccl_info): {nranks, device, version}
        from ncclCommCount / ncclCommCuDevice / ncclGetVersion; None on a
        communicator without RCCL."""
        n, d, v = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = coll().mvx_comm_rccl_info(self.handle, ctypes.byref(n), ctypes.byref(d), ctypes.byref(v))
        if rc:
            return None
        return {"nranks": n.value, "device": d.value, "version": v.value}

    def reserve(self, nbytes):
        return coll().mvx_comm_reserve(self.handle, nbytes)

    def set_exchange(self, mode, slices=0):
        """EXCH_P2P / EXCH_PIPE (with `slices`) / EXCH_COLL (mvx_comm_set_exchange)."""
        return coll().mvx_comm_set_exchange(self.handle, mode, slices)

    def get_exchange(self):
        m, s = ctypes.c_int(), ctypes.c_int()
        rc = coll().mvx_comm_get_exchange(self.handle, ctypes.byref(m), ctypes.byref(s))
        if rc:
            raise RuntimeError("mvx_comm_get_exchange rc=%d" % rc)
        return m.value, s.value

    def last_exchange(self):
        """The variant the last call ran (mvx_comm_last_exchange): EXCH_*,
        or -1 when it moved nothing between ranks."""
        m = ctypes.c_int()
        rc = coll().mvx_comm_last_exchange(self.handle, ctypes.byref(m))
        if rc:
            raise RuntimeError("mvx_comm_last_exchange rc=%d" % rc)
        return m.value

    def set_phase_timing(self, on=True):
        """Record HIP events around phases A / B / C of every device call
        (mvx_comm_set_phase_timing)."""
        return coll().mvx_comm_set_phase_timing(self.handle, 1 if on else 0)

    def phase_times(self):
        """{'A', 'B', 'C', 'total'} in ms of the last timed device call
        (None for a phase of the pipelined variant, whose phases overlap)."""
        ms = (ctypes.c_float * 4)()
        rc = coll().mvx_comm_phase_times(self.handle, ms)
        if rc:
            raise RuntimeError("mvx_comm_phase_times rc=%d" % rc)
        v = [None if x < 0 else round(float(x), 5) for x in ms]
        return {"A": v[0], "B": v[1], "C": v[2], "total": v[3]}

    def get_tuning(self):
        """The communicator's device flavour and knobs (a Tuning)."""
        from . import Tuning
        t = Tuning()
        rc = coll().mvx_comm_get_tuning(self.handle, ctypes.byref(t))
        if rc:
            raise RuntimeError("mvx_comm_get_tuning rc=%d" % rc)
        return t

    def set_tuning(self, tuning):
        return coll().mvx_comm_set_tuning(self.handle, ctypes.byref(tuning))

    # stream-ordered (device buffers)
    def allreduce_async(self, sendbuf, recvbuf, count, dtype, op, stream=None):
        return coll().mvx_allreduce_async(addr(sendbuf), addr(recvbuf), count, dtype, op, self.handle,
                                          stream_handle(stream))

    def reduce_async(self, sendbuf, recvbuf, count, dtype, op, root, stream=None):
        return coll().mvx_reduce_async(addr(sendbuf), addr(recvbuf), count, dtype, op, root, self.handle,
                                       stream_handle(stream))

    def scan_async(self, sendbuf, recvbuf, count, dtype, op, stream=None):
        return coll().mvx_scan_async(addr(sendbuf), addr(recvbuf), count, dtype, op, self.handle,
                                     stream_handle(stream))

    def scan_multi(self, sendbufs, recvbufs, count, dtype, op, stream=None):
        rc = (ctypes.c_int * self.size)()
        r = coll().mvx_scan_multi(_pp(sendbufs), _pp(recvbufs), count, dtype, op, self.handle, rc,
                                  stream_handle(stream))
        return r, list(rc)

    def reduce_scatter_async(self, sendbuf, recvbuf, recvcnts, dtype, op, stream=None):
        cn = (ctypes.c_int * len(recvcnts))(*recvcnts)
        return coll().mvx_reduce_scatter_async(addr(sendbuf), addr(recvbuf), cn, dtype, op, self.handle,
                                               stream_handle(stream))

    # virtual communicators: all ranks' buffers at once, per-rank codes back
    def allreduce_multi(self, sendbufs, recvbufs, count, dtype, op, stream=None):
        rc = (ctypes.c_int * self.size)()
        r = coll().mvx_allreduce_multi(_pp(sendbufs), _pp(recvbufs), count, dtype, op, self.handle, rc,
                                       stream_handle(stream))
        return r, list(rc)

    def reduce_multi(self, sendbufs, recvbufs, count, dtype, op, root, stream=None):
        rc = (ctypes.c_int * self.size)()
        r = coll().mvx_reduce_multi(_pp(sendbufs), _pp(recvbufs), count, dtype, op, root, self.handle, rc,
                                    stream_handle(stream))
        return r, list(rc)

    def reduce_scatter_multi(self, sendbufs, recvbufs, recvcnts, dtype, op, stream=None):
        rc = (ctypes.c_int * self.size)()
        cn = (ctypes.c_int * self.size)(*recvcnts)
        r = coll().mvx_reduce_scatter_multi(_pp(sendbufs), _pp(recvbufs), cn, dtype, op, self.handle, rc,
                                            stream_handle(stream))
        return r, list(rc)


def _comm_handle(comm):
    return comm.handle if isinstance(comm, Comm) else comm


# -------------------------------------------------------- MPI-named mirror

def MPI_Allreduce(sendbuf, recvbuf, count, datatype, op, comm):
    return coll().MPI_Allreduce(addr(sendbuf), addr(recvbuf), count, datatype, op, _comm_handle(comm))


def MPI_Reduce(sendbuf, recvbuf, count, datatype, op, root, comm):
    return coll().MPI_Reduce(addr(sendbuf), addr(recvbuf), count, datatype, op, root, _comm_handle(comm))


def MPI_Reduce_scatter(sendbuf, recvbuf, recvcnts, datatype, op, comm):
    cn = (ctypes.c_int * len(recvcnts))(*recvcnts) if recvcnts is not None else None
    return coll().MPI_Reduce_scatter(addr(sendbuf), addr(recvbuf), cn, datatype, op, _comm_handle(comm))


def MPI_Scan(sendbuf, recvbuf, count, datatype, op, comm):
    return coll().MPI_Scan(addr(sendbuf), addr(recvbuf), count, datatype, op, _comm_handle(comm))


_USER_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                            ctypes.POINTER(ctypes.c_int))
_keepalive = []


def MPI_Op_create(function, commute):
    """Returns (rc, op_handle).  `function` is a C MPI_User_function address
    (int) or a Python callable `function(invec, inoutvec, len_ptr, type_ptr)`."""
    if isinstance(function, int):
        fp = ctypes.c_void_p(function)
    else:
        cb = _USER_FN(function)
        _keepalive.append(cb)
        fp = ctypes.cast(cb, ctypes.c_void_p)
    h = ctypes.c_int()
    rc = coll().MPI_Op_create(fp, commute, ctypes.byref(h))
    return rc, h.value


def op_create_device(function_addr, commute):
    """mvx_op_create_device: `function_addr` is the address of a C
    MVX_Device_function (int (*)(const void *in, void *inout, size_t len,
    MPI_Datatype, void *stream)) that enqueues the op on `stream`.
    Returns (rc, op_handle)."""
    h = ctypes.c_int()
    rc = coll().mvx_op_create_device(ctypes.c_void_p(function_addr), commute, ctypes.byref(h))
    return rc, h.value


def MPI_Op_free(op):
    """Returns (rc, new_handle)."""
    h = ctypes.c_int(op)
    rc = coll().MPI_Op_free(ctypes.byref(h))
    return rc, h.value


def MPI_Type_contiguous(count, oldtype):
    """Returns (rc, new handle)."""
    h = ctypes.c_int()
    rc = coll().MPI_Type_contiguous(count, oldtype, ctypes.byref(h))
    return rc, h.value


def _iarr(vals, ct=ctypes.c_int):
    return (ct * max(len(vals), 1))(*vals)


def MPI_Type_vector(count, blocklen, stride, oldtype):
    """Returns (rc, new handle)."""
    h = ctypes.c_int()
    rc = coll().MPI_Type_vector(count, blocklen, stride, oldtype, ctypes.byref(h))
    return rc, h.value


def MPI_Type_hvector(count, blocklen, stride_bytes, oldtype):
    h = ctypes.c_int()
    rc = coll().MPI_Type_hvector(count, blocklen, stride_bytes, oldtype, ctypes.byref(h))
    return rc, h.value


def MPI_Type_indexed(count, blocklens, indices, oldtype):
    h = ctypes.c_int()
    rc = coll().MPI_Type_indexed(count, _iarr(blocklens), _iarr(indices), oldtype, ctypes.byref(h))
    return rc, h.value


def MPI_Type_hindexed(count, blocklens, byte_indices, oldtype):
    h = ctypes.c_int()
    rc = coll().MPI_Type_hindexed(count, _iarr(blocklens), _iarr(byte_indices, ctypes.c_long), oldtype,
                                  ctypes.byref(h))
    return rc, h.value


def MPI_Type_struct(count, blocklens, byte_indices, types):
    h = ctypes.c_int()
    rc = coll().MPI_Type_struct(count, _iarr(blocklens), _iarr(byte_indices, ctypes.c_long), _iarr(types),
                                ctypes.byref(h))
    return rc, h.value


def MPI_Type_lb(datatype):
    v = ctypes.c_long()
    rc = coll().MPI_Type_lb(datatype, ctypes.byref(v))
    return rc, v.value


def MPI_Type_ub(datatype):
    v = ctypes.c_long()
    rc = coll().MPI_Type_ub(datatype, ctypes.byref(v))
    return rc, v.value


def type_layout(datatype):
    """dict(kind, dense, lb, ub, span_lo, span_hi) from mvx_type_layout."""
    k, d = ctypes.c_int(), ctypes.c_int()
    lb, ub, lo, hi = ctypes.c_long(), ctypes.c_long(), ctypes.c_long(), ctypes.c_long()
    rc = hip().mvx_type_layout(datatype, ctypes.byref(k), ctypes.byref(d), ctypes.byref(lb), ctypes.byref(ub),
                               ctypes.byref(lo), ctypes.byref(hi))
    if rc:
        raise ValueError("mvx_type_layout rc=%d" % rc)
    return dict(kind=k.value, dense=d.value, lb=lb.value, ub=ub.value, span_lo=lo.value, span_hi=hi.value)


def type_set_handle(datatype, handle):
    """The handle user functions receive for `datatype` (mvx_type_set_handle,
    include/mvx_embed.h); handle == datatype removes the mapping."""
    return coll().mvx_type_set_handle(datatype, handle)


def type_pack(datatype, origin, packed, count, stream=None):
    return hip().mvx_type_pack(datatype, addr(origin), addr(packed), count, stream_handle(stream))


def type_unpack(datatype, packed, origin, count, stream=None):
    return hip().mvx_type_unpack(datatype, addr(packed), addr(origin), count, stream_handle(stream))


def MPI_Type_commit(datatype):
    h = ctypes.c_int(datatype)
    return coll().MPI_Type_commit(ctypes.byref(h))


def MPI_Type_free(datatype):
    """Returns (rc, new handle)."""
    h = ctypes.c_int(datatype)
    rc = coll().MPI_Type_free(ctypes.byref(h))
    return rc, h.value


def MPI_Type_extent(datatype):
    """Returns (rc, extent)."""
    e = ctypes.c_long()
    rc = coll().MPI_Type_extent(datatype, ctypes.byref(e))
    return rc, e.value


def MPI_Type_size(datatype):
    """Returns (rc, size)."""
    s = ctypes.c_int()
    rc = coll().MPI_Type_size(datatype, ctypes.byref(s))
    return rc, s.value


def MPIR_call(name, invec, inoutvec, length, datatype):
    """Call a predefined op through its MPI_User_function symbol (e.g. "MPIR_SUM")."""
    ln = ctypes.c_int(length)
    dt = ctypes.c_int(datatype)
    getattr(coll(), name)(addr(invec), addr(inoutvec), ctypes.byref(ln), ctypes.byref(dt))


def op_errno():
    return coll().mvx_op_errno()


def comm_reap():
    """mvx_comm_reap: free drained aborted communicators' staging; returns
    how many are still held."""
    return coll().mvx_comm_reap()


def host_register_enable(on=True, max_bytes=0):
    """The pageable-buffer registration cache (mvx_host_register_enable).

    A Python process loads libmvx.so with dlopen, so its release hooks are
    not the process's (mvx_host_hooks_active() is 0 here): the cache runs in
    mode 2, and the caller reports every release of a buffer it passed with
    host_unregister / host_invalidate before the memory is freed.  A C
    program linked with -lmvx gets mode 1, releases seen by the hooks."""
    mode = 0
    if on:
        mode = 1 if coll().mvx_host_hooks_active() else 2
    return coll().mvx_host_register_enable(mode, max_bytes)


def host_hooks_active():
    """mvx_host_hooks_active: libmvx.so's release hooks are the process's."""
    return bool(coll().mvx_host_hooks_active())


def host_invalidate(address, nbytes):
    """mvx_host_invalidate: drop registrations overlapping [address,
    address + nbytes), about to be released; returns how many."""
    return coll().mvx_host_invalidate(address, nbytes)


def host_unregister(buf):
    """mvx_host_unregister: drop the registrations containing buf's address
    (call before freeing a registered buffer)."""
    return coll().mvx_host_unregister(addr(buf))


def host_register_stats():
    """{entries, bytes, hits, misses} of the registration cache."""
    e, b, h, m = ctypes.c_long(), ctypes.c_size_t(), ctypes.c_long(), ctypes.c_long()
    coll().mvx_host_register_stats(ctypes.byref(e), ctypes.byref(b), ctypes.byref(h), ctypes.byref(m))
    return {"entries": e.value, "bytes": b.value, "hits": h.value, "misses": m.value}


def host_register_deferred():
    """{deferred, held, unregisters, bounced}: registrations a release
    dropped that are not unregistered yet (a call still holds them, or no
    libmvx entry has run since), registrations held by calls in flight, the
    hipHostUnregister calls made so far, and ranges copied through the CPU
    because another call's registration covered part of their pages
    (mvx_host_register_deferred)."""
    d, h, u, b = ctypes.c_long(), ctypes.c_long(), ctypes.c_long(), ctypes.c_long()
    coll().mvx_host_register_deferred(ctypes.byref(d), ctypes.byref(h), ctypes.byref(u), ctypes.byref(b))
    return {"deferred": d.value, "held": h.value, "unregisters": u.value, "bounced": b.value}
