"""A host transport for libmvx.so communicators (mvx_comm_init_transport).

The product's multi-GPU transport is RCCL over xGMI (mvx_comm_init).  This
module supplies the other kind the C executor accepts: a caller-side byte
mover, here torch.distributed point-to-point over any backend (gloo on the
host).  With it several processes can share one GPU as separate ranks --
RCCL refuses that ("Duplicate GPU detected") -- and run exactly the plan,
phase and combine code of the RCCL path, only the bytes between ranks travel
through host memory.  The executor's contract (include/mvx_coll.h): a phase
is start, sends / receives, end; end returns once received bytes are in
place; sends and receives between a pair of ranks pair up in call order.
"""
import ctypes

from . import coll

_START = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
_XFER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                         ctypes.c_void_p)
_END = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)


class Transport(ctypes.Structure):
    """Mirror of ``mvx_transport``."""
    _fields_ = [("ctx", ctypes.c_void_p), ("start", _START), ("send", _XFER), ("recv", _XFER), ("end", _END)]


class TorchP2PTransport:
    """Phases as torch.distributed isend / irecv of host copies."""

    def __init__(self, group=None):
        self.group = group
        self.pending = []
        self.errors = []
        self._c = Transport(None, _START(self._start), _XFER(self._send), _XFER(self._recv), _END(self._end))

    def struct(self):
        return self._c

    def _start(self, ctx):
        self.pending = []
        return 0

    def _send(self, ctx, buf, nbytes, peer, stream):
        self.pending.append((True, buf, nbytes, peer))
        return 0

    def _recv(self, ctx, buf, nbytes, peer, stream):
        self.pending.append((False, buf, nbytes, peer))
        return 0

    def _end(self, ctx, stream):
        try:
            import torch
            import torch.distributed as dist
            L = coll()
            if L.mvx_stream_synchronize(stream):
                return 1
            reqs, landing = [], []
            for is_send, buf, nbytes, peer in self.pending:
                host = torch.empty(nbytes, dtype=torch.uint8)
                if is_send:
                    if L.mvx_copy(host.data_ptr(), buf, nbytes):
                        return 1
                    reqs.append(dist.isend(host, dst=peer, group=self.group))
                else:
                    reqs.append(dist.irecv(host, src=peer, group=self.group))
                    landing.append((buf, host, nbytes))
            for r in reqs:
                r.wait()
            for buf, host, nbytes in landing:
                if L.mvx_copy(buf, host.data_ptr(), nbytes):
                    return 1
            self.pending = []
            return 0
        except Exception as e:          # a callback must not raise into C
            self.errors.append(repr(e))
            return 1
