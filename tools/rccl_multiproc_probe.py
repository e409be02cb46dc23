#!/usr/bin/env python3
"""Probe: can p processes share the one GPU of the test box as p RCCL ranks?

If RCCL accepts it, the exact N > 1 executor (mvx_comm_init + RCCL grouped
send/recv + combine kernels) runs here against the oracle's replay; if it
refuses (duplicate GPU), every rank reports the RCCL error and exits 0.
Test infrastructure: processes are spawned fresh (no GPU state inherited).
"""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, out):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import importlib

    import numpy as np
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    mvx = importlib.import_module("mvapich-cce_amd")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    try:
        comm = mvx.Comm.from_torch_distributed(0)
    except Exception as e:     # RCCL refused: report and stop
        res["init"] = str(e)
        dist.barrier()
        with open(os.path.join(out, "r%d.json" % rank), "w") as f:
            json.dump(res, f)
        return
    res["init"] = "ok"
    fails = []
    for (n, dt, op) in ((1000, 10, 102), (70001, 10, 102), (1 << 20, 10, 102), (5000, 17, 111), (30000, 8, 105)):
        npdt = mvx.NP_DTYPE[dt]
        sends = []
        for r in range(world):
            a = np.zeros(n, npdt)
            O.fill(a, n, 4 if dt == 17 else (2 if dt == 8 else 0), r)
            sends.append(a)
        ref = [np.zeros_like(sends[0]) for _ in range(world)]
        O.allreduce([s.view(np.uint8) for s in sends], [x.view(np.uint8) for x in ref], n, dt, op)
        d = torch.from_numpy(sends[rank].view(np.uint8).copy()).cuda()
        o = torch.zeros_like(d)
        rc = mvx.MPI_Allreduce(d, o, n, dt, op, comm)
        got = o.cpu().numpy()
        if rc or not np.array_equal(got, ref[rank].view(np.uint8)):
            fails.append((n, dt, op, rc))
    res["fails"] = fails
    comm.free()
    dist.barrier()
    with open(os.path.join(out, "r%d.json" % rank), "w") as f:
        json.dump(res, f)


def main():
    import tempfile

    import torch.multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    out = tempfile.mkdtemp()
    mp.spawn(worker, args=(world, _port(), out), nprocs=world, join=True)
    for r in range(world):
        with open(os.path.join(out, "r%d.json" % r)) as f:
            print(f.read())


if __name__ == "__main__":
    main()
