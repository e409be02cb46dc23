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
The optional alltoall / allgather hooks carry the MVX_EXCH_COLL variant
(what ncclAllToAll / ncclAllGather do on the RCCL path) as gloo
all_to_all_single / all_gather.
"""
import ctypes

from . import coll

_START = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
_XFER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                         ctypes.c_void_p)
_END = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
_A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                        ctypes.c_void_p)
_AG = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


def rccl_net_env(rank, env=None):
    """Make RCCL itself carry the bytes between ranks that share one GPU.

    RCCL's duplicate-GPU check compares (host hash, PCI bus id) of every
    pair of ranks; the host hash is NCCL_HOSTID when that is set.  Giving
    each rank its own host id makes them separate one-GPU "nodes", so RCCL
    accepts the communicator and moves every byte through its network
    transport (sockets over loopback, host-staged by its proxy thread):
    the RCCL calls of the executor (grouped ncclSend / ncclRecv,
    ncclAllToAll, in-place ncclAllGather, ncclCommAbort) run for real at
    p > 1 on a one-GPU box.  Not a performance configuration -- on a node
    every rank has its own GPU and RCCL picks xGMI P2P.  Must run before
    the process's first RCCL call.  Returns the environment it changed."""
    import os
    env = os.environ if env is None else env
    env["NCCL_HOSTID"] = "mvx-rank-%d" % rank
    env.setdefault("NCCL_SOCKET_IFNAME", "lo")
    env.setdefault("NCCL_IB_DISABLE", "1")
    return env


class Transport(ctypes.Structure):
    """Mirror of ``mvx_transport``."""
    _fields_ = [("ctx", ctypes.c_void_p), ("start", _START), ("send", _XFER), ("recv", _XFER), ("end", _END),
                ("alltoall", _A2A), ("allgather", _AG)]


class TorchP2PTransport:
    """Phases as torch.distributed isend / irecv of host copies; with
    `collectives` (default) also the alltoall / allgather hooks."""

    def __init__(self, group=None, collectives=True):
        self.group = group
        self.pending = []
        self.errors = []
        a2a = _A2A(self._alltoall) if collectives else _A2A()
        ag = _AG(self._allgather) if collectives else _AG()
        self._c = Transport(None, _START(self._start), _XFER(self._send), _XFER(self._recv), _END(self._end),
                            a2a, ag)

    def struct(self):
        return self._c

    def _peer(self, peer):
        """libmvx passes communicator ranks; torch.distributed's dst / src
        are global ranks even when a group is given"""
        if self.group is None:
            return peer
        import torch.distributed as dist
        return dist.get_global_rank(self.group, peer)

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
                    reqs.append(dist.isend(host, dst=self._peer(peer), group=self.group))
                else:
                    reqs.append(dist.irecv(host, src=self._peer(peer), group=self.group))
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

    def _alltoall(self, ctx, sendbuf, recvbuf, nbytes, stream):
        try:
            import torch
            import torch.distributed as dist
            L = coll()
            if L.mvx_stream_synchronize(stream):
                return 1
            p = dist.get_world_size(self.group)
            src = torch.empty(p * nbytes, dtype=torch.uint8)
            dst = torch.empty(p * nbytes, dtype=torch.uint8)
            if L.mvx_copy(src.data_ptr(), sendbuf, p * nbytes):
                return 1
            dist.all_to_all_single(dst, src, group=self.group)
            if L.mvx_copy(recvbuf, dst.data_ptr(), p * nbytes):
                return 1
            return 0
        except Exception as e:
            self.errors.append(repr(e))
            return 1

    def _allgather(self, ctx, buf, nbytes, stream):
        try:
            import torch
            import torch.distributed as dist
            L = coll()
            if L.mvx_stream_synchronize(stream):
                return 1
            p = dist.get_world_size(self.group)
            me = dist.get_rank(self.group)
            mine = torch.empty(nbytes, dtype=torch.uint8)
            if L.mvx_copy(mine.data_ptr(), buf + me * nbytes, nbytes):
                return 1
            parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(p)]
            dist.all_gather(parts, mine, group=self.group)
            for j in range(p):      # in place: this rank's block is already there
                if j != me and L.mvx_copy(buf + j * nbytes, parts[j].data_ptr(), nbytes):
                    return 1
            return 0
        except Exception as e:
            self.errors.append(repr(e))
            return 1
