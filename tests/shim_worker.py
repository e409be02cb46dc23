#!/usr/bin/env python3
"""TEST HELPER: one rank of the MVAPICH collops shim (integration/intra_mvx.c)
in a multi-process world (integration/check/harness.c h_init_world).

  shim_worker.py RANK NP BOARD OUT.json SCENARIO

Every rank builds every rank's inputs from seeds and checks its own result
against the oracle's replay of the reference schedule over all of them.
Scenarios:
  route      host buffers on every rank: MVAPICH's own path on every rank,
             one route agreement per call; none for an empty call, none
             under MVX_SHIM_ROUTE=local
  want       the caller's environment decides each rank's wish (the test
             sets MVX_HOST_BUFFERS=1 on some ranks); host buffers; every
             rank reports each call's code and elapsed time
  mixed      rank 0 device buffers, the others host buffers (GPU,
             RCCL over its socket transport): every rank through libmvx,
             bit-exact against the oracle, for the four collectives
  fail       as `mixed`; the caller's MVX_DEVICE_ID makes one rank's device
             unusable: every rank returns an error, none hangs
Writes a JSON report.
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE]

FLOAT, INT = 10, 6
MPI_SUM, MPI_MAX = 102, 100
COLL_ALLREDUCE, COLL_REDUCE, COLL_REDUCE_SCATTER, COLL_SCAN = 0, 1, 2, 3


def main():
    rank, world, board, out, scenario = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                         sys.argv[5])
    import numpy as np

    from oracle import oracle as O
    from test_cpu_integration import Nodes, _lib

    gpu = scenario in ("mixed", "fail")
    if gpu:
        import importlib
        importlib.import_module("mvapich-cce_amd.transport").rccl_net_env(rank)
    lib = _lib(init=False)
    lib.h_init_world.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_double]
    assert lib.h_init_world(rank, world, board.encode(), 90.0) == 0
    N = Nodes(lib, O)
    fh, fnode = N.basic(FLOAT)
    rep = {"rank": rank, "calls": [], "fails": []}

    def call(name, fn):
        a0, h0 = lib.h_agree_calls(), lib.h_host_calls()
        t0 = time.time()
        rc = fn()
        rep["calls"].append({"name": name, "rc": rc, "s": round(time.time() - t0, 3),
                             "agree": lib.h_agree_calls() - a0, "host": lib.h_host_calls() - h0})
        return rc

    n = 1000
    sends = [np.arange(n, dtype=np.float32) * (r + 1) + 0.25 * r for r in range(world)]

    if scenario in ("route", "want"):
        s = sends[rank]
        r = np.zeros(n, np.float32)
        cn = (ctypes.c_int * world)(*([n // world] * world))
        call("allreduce", lambda: lib.h_allreduce(s.ctypes.data, r.ctypes.data, n, fnode, MPI_SUM))
        call("reduce", lambda: lib.h_reduce(s.ctypes.data, r.ctypes.data, n, fnode, MPI_SUM, 0))
        call("reduce_scatter", lambda: lib.h_reduce_scatter(s.ctypes.data, r.ctypes.data, cn, fnode, MPI_SUM))
        call("scan", lambda: lib.h_scan(s.ctypes.data, r.ctypes.data, n, fnode, MPI_SUM))
        call("allreduce_again", lambda: lib.h_allreduce(s.ctypes.data, r.ctypes.data, n, fnode, MPI_SUM))
        if scenario == "route":
            call("empty", lambda: lib.h_allreduce(s.ctypes.data, r.ctypes.data, 0, fnode, MPI_SUM))
            os.environ["MVX_SHIM_ROUTE"] = "local"
            call("local", lambda: lib.h_allreduce(s.ctypes.data, r.ctypes.data, n, fnode, MPI_SUM))
            del os.environ["MVX_SHIM_ROUTE"]
    else:
        import torch
        torch.cuda.set_device(0)
        dev = rank == 0

        def buf(a):
            return torch.from_numpy(a.copy()).cuda() if dev else a.copy()

        def ptr(b):
            return b.data_ptr() if dev else b.ctypes.data

        def host(b):
            return b.cpu().numpy() if dev else b

        cnts = [n // world + (1 if q < n % world else 0) for q in range(world)]
        cases = [("allreduce", COLL_ALLREDUCE), ("reduce", COLL_REDUCE), ("reduce_scatter", COLL_REDUCE_SCATTER),
                 ("scan", COLL_SCAN)]
        for name, coll in cases:
            nrecv = cnts[rank] if coll == COLL_REDUCE_SCATTER else n
            s = buf(sends[rank])
            r = buf(np.full(nrecv, -7.0, np.float32))
            cn = (ctypes.c_int * world)(*cnts)
            root = world - 1
            if coll == COLL_ALLREDUCE:
                rc = call(name, lambda: lib.h_allreduce(ptr(s), ptr(r), n, fnode, MPI_SUM))
            elif coll == COLL_REDUCE:
                rc = call(name, lambda: lib.h_reduce(ptr(s), ptr(r), n, fnode, MPI_SUM, root))
            elif coll == COLL_REDUCE_SCATTER:
                rc = call(name, lambda: lib.h_reduce_scatter(ptr(s), ptr(r), cn, fnode, MPI_SUM))
            else:
                rc = call(name, lambda: lib.h_scan(ptr(s), ptr(r), n, fnode, MPI_SUM))
            if scenario == "fail":
                continue
            if dev:
                torch.cuda.synchronize()
            got = host(r)
            exp = [np.full(cnts[q] if coll == COLL_REDUCE_SCATTER else n, -7.0, np.float32) for q in range(world)]
            bs = [x.view(np.uint8) for x in sends]
            be = [x.view(np.uint8) for x in exp]
            if coll == COLL_ALLREDUCE:
                O.allreduce(bs, be, n, FLOAT, MPI_SUM)
            elif coll == COLL_REDUCE:
                O.reduce(bs, be, n, FLOAT, MPI_SUM, root)
            elif coll == COLL_REDUCE_SCATTER:
                O.reduce_scatter(bs, be, cnts, FLOAT, MPI_SUM)
            else:
                O.scan(bs, be, n, FLOAT, MPI_SUM)
            if coll == COLL_REDUCE and rank != root:
                continue                      # recvbuf is significant at the root only
            if rc != 0 or not np.array_equal(got.view(np.uint32), exp[rank].view(np.uint32)):
                rep["fails"].append({"case": name, "rc": rc})
    with open(out, "w") as f:
        json.dump(rep, f)


if __name__ == "__main__":
    main()
