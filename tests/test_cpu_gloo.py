"""CPU, multi-process: the N > 1 path's host logic over a real process group.

Each process is one rank (torch.distributed, gloo, 127.0.0.1).  It builds
its own plan with libmvx.so (exactly what the RCCL executor runs), moves the
phase A / phase C ranges with gloo point-to-point messages (the role RCCL
send/recv plays on the GPUs), evaluates its phase B combine with the oracle
op, and checks its own result against the oracle's replay of the reference
schedule.  This is the distributed path minus the device kernels, which the
-m gpu tests cover.
"""
import importlib
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


CASES = [  # (coll, count, dtype, op, root)
    (1, 10, 6, 102, 0), (1, 5000, 10, 102, 0), (1, 70001, 10, 102, 0), (1, 3000, 10, 100, 0),
    (1, 40000, 17, 111, 0), (1, 20000, 8, 105, 0), (1, 9, 18, 110, 0),
    (2, 10, 6, 102, 0), (2, 30000, 10, 102, 1), (2, 30000, 11, 101, 0), (2, 5000, 17, 110, 1),
    (3, 7, 6, 102, 0), (3, 200, 10, 102, 0), (3, 60000, 10, 102, 0), (3, 60000, 8, 105, 0),
    (3, 5000, 17, 111, 0), (4, 10, 6, 102, 0), (4, 3000, 10, 102, 0), (4, 700, 17, 110, 0),
    # user ops (tests/user_ops.c): "name:commute"
    (1, 3000, 7, "mix:0", 0), (1, 3000, 7, "mix:1", 0), (2, 2000, 9, "affine:0", 1),
    (3, 20, 7, "mix:0", 0), (3, 300, 7, "mix:0", 0), (4, 500, 9, "affine:0", 0), (3, 300, 10, "fsum:1", 0),
]


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, HERE]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import mvxtest as T
    import uops
    from oracle import oracle as O
    from plan_exec import run_plan_program

    mvx = importlib.import_module("mvapich-cce_amd")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    failures = []
    for ci, (coll, n, dtype, op, root) in enumerate(CASES):
        cnts = [n + (r % 3) for r in range(world)] if coll == 3 else None
        tot = sum(cnts) if cnts else n
        kind = None
        if isinstance(op, str):
            name, commute = op.split(":")
            op, kind = 250, (1 if commute == "1" else 2)
            O.user_op_set(op, uops.host_fn(name), int(commute))
            S = [uops.rand_for(name, tot, 1000 * ci + r) for r in range(world)]
        else:
            S = [T.rand_vec(dtype, tot, 1000 * ci + r) for r in range(world)]
        E = S[0].dtype.itemsize
        sb = [s.view(np.uint8) for s in S]
        # oracle: the reference schedule over all ranks
        if coll == 1:
            R0 = [np.zeros_like(S[0]) for _ in range(world)]
            O.allreduce(sb, [x.view(np.uint8) for x in R0], n, dtype, op)
            mine = R0[rank]
            recvbuf = np.zeros(tot * E, np.uint8)
        elif coll == 2:
            R0 = [np.zeros_like(S[0]) for _ in range(world)]
            O.reduce(sb, [x.view(np.uint8) for x in R0], n, dtype, op, root)
            mine = R0[rank] if rank == root else None
            recvbuf = np.zeros(tot * E, np.uint8)
        elif coll == 4:
            R0 = [np.zeros_like(S[0]) for _ in range(world)]
            O.scan(sb, [x.view(np.uint8) for x in R0], n, dtype, op)
            mine = R0[rank]
            recvbuf = np.zeros(tot * E, np.uint8)
        else:
            R0 = [np.zeros(max(c, 1), S[0].dtype) for c in cnts]
            O.reduce_scatter(sb, [x.view(np.uint8) for x in R0], cnts, dtype, op)
            mine = R0[rank][: cnts[rank]]
            recvbuf = np.zeros(max(cnts[rank], 1) * E, np.uint8)
        P = mvx.plan(coll, world, rank, n, dtype, op, root, cnts, opkind=kind)
        send = sb[rank]
        # phase A
        reqs, slot = [], {}
        for s in range(world):
            if P.a_send[s].cnt:
                o, c = P.a_send[s].off * E, P.a_send[s].cnt * E
                reqs.append(dist.isend(torch.from_numpy(send[o:o + c].copy()), dst=s, tag=1))
            if P.a_recv[s].cnt:
                slot[s] = torch.empty(P.a_recv[s].cnt * E, dtype=torch.uint8)
                reqs.append(dist.irecv(slot[s], src=s, tag=1))
        for q in reqs:
            q.wait()
        # phase B
        out = None
        if P.has_combine and P.c_cnt:
            lo, hi = P.c_src_off * E, (P.c_src_off + P.c_cnt) * E

            def leaf(s):
                return send[lo:hi] if s == rank else slot[s].numpy()
            leaves = [leaf(P.leaf[q]) for q in range(P.k)]
            folds = [leaf(P.leaf_fold[q]) if P.leaf_fold[q] >= 0 else None for q in range(P.k)]
            out = run_plan_program(P, leaves, folds, P.c_cnt)
            if not P.c_dst_tmp:
                recvbuf[P.c_dst_off * E: P.c_dst_off * E + out.size] = out
        # phase C
        reqs = []
        for s in range(world):
            if P.b_send[s].cnt:
                reqs.append(dist.isend(torch.from_numpy(out[: P.b_send[s].cnt * E].copy()), dst=s, tag=2))
            if P.b_recv[s].cnt:
                buf = torch.empty(P.b_recv[s].cnt * E, dtype=torch.uint8)
                reqs.append((dist.irecv(buf, src=s, tag=2), buf, P.b_recv[s].off * E))
        for q in reqs:
            if isinstance(q, tuple):
                q[0].wait()
                recvbuf[q[2]: q[2] + q[1].numel()] = q[1].numpy()
            else:
                q.wait()
        if mine is not None:
            try:
                if kind is not None:
                    assert np.array_equal(recvbuf[: mine.nbytes], mine.view(np.uint8)), "user op result differs"
                else:
                    T.assert_same(op, dtype, recvbuf[: mine.nbytes], mine, typemap_only=True)
            except AssertionError as e:
                failures.append("case %d rank %d: %s" % (ci, rank, e))
        dist.barrier()
    dist.destroy_process_group()
    with open(os.path.join(out_dir, "rank%d.txt" % rank), "w") as f:
        f.write("\n".join(failures))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_plans_over_gloo(tmp_path, world):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        txt = (tmp_path / ("rank%d.txt" % r)).read_text()
        assert txt == "", txt


def _peer_worker(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, HERE]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    tp = importlib.import_module("mvapich-cce_amd.transport")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = dist.new_group([1, 2])
    got = []
    if rank in (1, 2):
        t = tp.TorchP2PTransport(group=g)
        got = [t._peer(0), t._peer(1)]
    assert tp.TorchP2PTransport()._peer(2) == 2
    dist.barrier()
    dist.destroy_process_group()
    with open(os.path.join(out_dir, "peer%d.txt" % rank), "w") as f:
        f.write(repr(got))


def test_transport_maps_group_ranks_to_global(tmp_path):
    """libmvx passes communicator ranks to the transport; with a sub-group,
    TorchP2PTransport sends to and receives from the matching global ranks
    (torch.distributed's dst / src are global even when a group is given)."""
    import torch.multiprocessing as mp
    mp.spawn(_peer_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)
    assert (tmp_path / "peer0.txt").read_text() == "[]"
    assert (tmp_path / "peer1.txt").read_text() == "[1, 2]"
    assert (tmp_path / "peer2.txt").read_text() == "[1, 2]"
