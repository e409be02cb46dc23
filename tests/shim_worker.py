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
  kinds_cpu  buffer kinds mixed within a rank (no GPU: the harness is told
             which host arrays to treat as device memory): every rank
             reports each call's route agreement -- this rank's ints and the
             reduced ones -- for the within-rank cases below
  kinds      the within-rank cases on the GPU (RCCL over its socket
             transport), bit-exact against the oracle at two sizes (the
             larger one sliced: MVX_SLICE_MIN_MIB=1 from the test):
               reduce_dh    device sendbuf everywhere, host recvbuf (the
                            non-roots' recvbuf is ignored)
               allreduce_dh device sendbuf, host recvbuf, on every rank
               rs_hd        rank 0 host sendbuf + device recvbuf, the other
                            ranks device buffers
               reduce_dd    device buffers everywhere (non-roots pass a host
                            recvbuf, which the call never touches)
               scan_dh      device sendbufs, host recvbufs on every rank
                            but the last
  latency    an 8-byte device Allreduce (two floats) 300 times with the route
             agreed and 300 times under MVX_SHIM_ROUTE=local (no agreement),
             interleaved in blocks; reports each mode's median call time
  xlate      MVX_HOST_BUFFERS=1 on every rank (from the test), a derived
             type whose node on rank 1 does not rebuild to the reference's
             bounds: every rank returns MPI_ERR_TYPE after the one route
             agreement, without creating the twin
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

    gpu = scenario in ("mixed", "fail", "kinds", "latency")
    if gpu:
        import importlib
        importlib.import_module("mvapich-cce_amd.transport").rccl_net_env(rank)
    lib = _lib(init=False)
    lib.h_init_world.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_double]
    lib.h_fake_device.argtypes = [ctypes.c_void_p, ctypes.c_long]
    lib.h_last_route.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    assert lib.h_init_world(rank, world, board.encode(), 90.0) == 0
    N = Nodes(lib, O)
    fh, fnode = N.basic(FLOAT)
    rep = {"rank": rank, "calls": [], "fails": []}

    def call(name, fn):
        a0, h0 = lib.h_agree_calls(), lib.h_host_calls()
        mine, alls = (ctypes.c_int * 3)(), (ctypes.c_int * 3)()
        r0 = lib.h_last_route(mine, alls)
        t0 = time.time()
        rc = fn()
        rec = {"name": name, "rc": rc, "s": round(time.time() - t0, 3),
               "agree": lib.h_agree_calls() - a0, "host": lib.h_host_calls() - h0}
        if lib.h_last_route(mine, alls) != r0:
            rec["route_mine"], rec["route_all"] = list(mine), list(alls)
        rep["calls"].append(rec)
        return rc

    n = 1000
    sends = [np.arange(n, dtype=np.float32) * (r + 1) + 0.25 * r for r in range(world)]

    if scenario == "xlate":
        from test_cpu_integration import DOUBLE
        i_, d_ = N.basic(INT), N.basic(DOUBLE)
        oh, good = N.struct([1, 1], [0, 8], [i_, d_])
        rc_, lb, ub, ext, size = O.type_bounds(oh)
        node = good if rank != 1 else lib.h_struct(2, (ctypes.c_int * 2)(1, 1), (ctypes.c_long * 2)(0, 8),
                                                   (ctypes.c_void_p * 2)(i_[1], d_[1]), lb, ub + 8, ext + 8, size)
        s = np.zeros(n * 16, np.uint8)
        r = np.zeros(n * 16, np.uint8)
        call("allreduce_bad_type", lambda: lib.h_allreduce(s.ctypes.data, r.ctypes.data, n, node, MPI_SUM))
        call("allreduce_good_type", lambda: lib.h_allreduce(s.ctypes.data, r.ctypes.data, n, good, MPI_SUM))
    elif scenario == "kinds_cpu":
        root = world - 1
        cn = (ctypes.c_int * world)(*([n // world] * world))

        def arr(k):
            return np.zeros(k, np.float32)

        def dev(a):
            assert lib.h_fake_device(a.ctypes.data, a.nbytes) == 0
            return a
        # device sendbuf everywhere, host recvbuf (the non-roots' ignored)
        s, r = dev(arr(n)), arr(n)
        call("reduce_dh", lambda: lib.h_reduce(s.ctypes.data, r.ctypes.data, n, fnode, MPI_SUM, root))
        # device sendbuf + host recvbuf on every rank
        s2, r2 = dev(arr(n)), arr(n)
        call("allreduce_dh", lambda: lib.h_allreduce(s2.ctypes.data, r2.ctypes.data, n, fnode, MPI_SUM))
        # rank 0: host sendbuf + device recvbuf; others device
        s3 = arr(n) if rank == 0 else dev(arr(n))
        r3 = dev(arr(n))
        call("rs_hd", lambda: lib.h_reduce_scatter(s3.ctypes.data, r3.ctypes.data, cn, fnode, MPI_SUM))
        # device everywhere; the non-roots' host recvbuf is never touched
        s4 = dev(arr(n))
        r4 = dev(arr(n)) if rank == root else arr(n)
        call("reduce_dd", lambda: lib.h_reduce(s4.ctypes.data, r4.ctypes.data, n, fnode, MPI_SUM, root))
        # device everywhere, Allreduce
        call("allreduce_dd", lambda: lib.h_allreduce(s4.ctypes.data, r3.ctypes.data, n, fnode, MPI_SUM))
    elif scenario == "latency":
        import torch
        torch.cuda.set_device(0)
        ds = torch.ones(2, dtype=torch.float32, device="cuda")
        dr = torch.zeros(2, dtype=torch.float32, device="cuda")
        times = {"agree": [], "local": []}
        for blk in range(12):
            for mode in ("agree", "local"):
                if mode == "local":
                    os.environ["MVX_SHIM_ROUTE"] = "local"
                for _ in range(25):
                    t0 = time.perf_counter()
                    rc = lib.h_allreduce(ds.data_ptr(), dr.data_ptr(), 2, fnode, MPI_SUM)
                    times[mode].append(time.perf_counter() - t0)
                    if rc:
                        rep["fails"].append({"case": "latency " + mode, "rc": rc})
                os.environ.pop("MVX_SHIM_ROUTE", None)
        if blk == 11 and float(dr[0]) != world:
            rep["fails"].append({"case": "latency value", "got": float(dr[0])})
        times = {k: sorted(v[5:]) for k, v in times.items()}      # the first calls create the twin
        rep["latency_us"] = {k: round(1e6 * v[len(v) // 2], 1) for k, v in times.items()}
    elif scenario == "kinds":
        import torch
        torch.cuda.set_device(0)
        root = world - 1

        def mk(a, on_dev):
            return torch.from_numpy(a.copy()).cuda() if on_dev else a.copy()

        def ptr(b):
            return b.data_ptr() if isinstance(b, torch.Tensor) else b.ctypes.data

        def host(b):
            return b.cpu().numpy() if isinstance(b, torch.Tensor) else b

        for size in (1000, 300001):
            S = [np.arange(size, dtype=np.float32) * (q + 1) + 0.25 * q for q in range(world)]
            cnts = [size // world + (1 if q < size % world else 0) for q in range(world)]
            # (name, coll, send on device, recv on device) for this rank
            cases = [("reduce_dh", COLL_REDUCE, True, False), ("allreduce_dh", COLL_ALLREDUCE, True, False),
                     ("rs_hd", COLL_REDUCE_SCATTER, rank != 0, True),
                     ("reduce_dd", COLL_REDUCE, True, rank == root),
                     ("scan_dh", COLL_SCAN, True, rank != root)]
            for name, coll, sd, rd in cases:
                nrecv = cnts[rank] if coll == COLL_REDUCE_SCATTER else size
                s = mk(S[rank], sd)
                r = mk(np.full(nrecv, -7.0, np.float32), rd)
                cn = (ctypes.c_int * world)(*cnts)
                tag = "%s %d" % (name, size)
                if coll == COLL_ALLREDUCE:
                    rc = call(tag, lambda: lib.h_allreduce(ptr(s), ptr(r), size, fnode, MPI_SUM))
                elif coll == COLL_REDUCE:
                    rc = call(tag, lambda: lib.h_reduce(ptr(s), ptr(r), size, fnode, MPI_SUM, root))
                elif coll == COLL_SCAN:
                    rc = call(tag, lambda: lib.h_scan(ptr(s), ptr(r), size, fnode, MPI_SUM))
                else:
                    rc = call(tag, lambda: lib.h_reduce_scatter(ptr(s), ptr(r), cn, fnode, MPI_SUM))
                torch.cuda.synchronize()
                exp = [np.full(cnts[q] if coll == COLL_REDUCE_SCATTER else size, -7.0, np.float32)
                       for q in range(world)]
                bs = [x.view(np.uint8) for x in S]
                be = [x.view(np.uint8) for x in exp]
                if coll == COLL_ALLREDUCE:
                    O.allreduce(bs, be, size, FLOAT, MPI_SUM)
                elif coll == COLL_REDUCE:
                    O.reduce(bs, be, size, FLOAT, MPI_SUM, root)
                elif coll == COLL_SCAN:
                    O.scan(bs, be, size, FLOAT, MPI_SUM)
                else:
                    O.reduce_scatter(bs, be, cnts, FLOAT, MPI_SUM)
                if coll == COLL_REDUCE and rank != root:
                    ok = rc == 0
                else:
                    ok = rc == 0 and np.array_equal(host(r).view(np.uint32), exp[rank].view(np.uint32))
                if not ok:
                    rep["fails"].append({"case": tag, "rc": rc})
    elif scenario in ("route", "want"):
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
