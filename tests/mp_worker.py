#!/usr/bin/env python3
"""TEST HELPER: one rank of a multi-process collective test.

Launched once per rank by tests/test_gpu_multiproc.py (fresh processes, no
GPU state inherited).  Every rank builds every rank's inputs from seeds, runs
the collectives through its libmvx.so communicator and compares its own
result with the oracle's replay of the reference schedule
(oracle/coll_sim.c) computed over all ranks' inputs.  Writes a JSON report.

  mp_worker.py RANK WORLD PORT OUT.json TRANSPORT(host|rccl|rccl-net) SUITE(small|random|full|mixed|sliced|graph)

rccl-net: RCCL communicators whose ranks may share one GPU, the bytes moved
by RCCL's own socket transport (transport.rccl_net_env).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE]


def main():
    import faulthandler
    faulthandler.enable()           # a crash in native code names the Python line it came from
    if os.environ.get("MVX_SEGV_BT") == "1":      # ... and the native frames (tools/segv_bt.c)
        import ctypes
        ctypes.CDLL(os.path.join(ROOT, "tools", "libsegv_bt.so")).segv_bt_install()
    rank, world, port, out, transport, suite = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                                 sys.argv[5], sys.argv[6])
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import importlib

    import numpy as np
    import torch
    import torch.distributed as dist

    import mvxtest as T
    from oracle import oracle as O
    mvx = importlib.import_module("mvapich-cce_amd")
    from importlib import import_module

    tp = import_module("mvapich-cce_amd.transport")
    if transport == "rccl-net":
        tp.rccl_net_env(rank)
    ndev = torch.cuda.device_count()
    dev = rank % ndev if transport != "rccl" else rank
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if transport == "host":
        comm = mvx.Comm.from_transport(tp.TorchP2PTransport(), dev)
    else:
        comm = mvx.Comm.from_torch_distributed(dev)
    report = {"rank": rank, "checked": 0, "fails": [], "ran": {}}

    def inputs(dtype, tot, fill):
        if fill is None:
            return [T.rand_vec(dtype, tot, 1000 * world + 17 * r + tot + dtype) for r in range(world)]
        out = []
        for r in range(world):          # SURVEY.md 8(d) distributions (oracle/cpu_ops.c orc_fill)
            a = np.empty(tot, T.np_dtype(dtype))
            O.fill(a, tot, fill, r)
            out.append(a)
        return out

    def check(coll, dtype, op, n_or_cnts, where, root=0, tag="", fill=None):
        E = mvx.dtype_info(dtype)[0]
        cnts = n_or_cnts if coll == "rs" else None
        tot = sum(cnts) if cnts else n_or_cnts
        S = inputs(dtype, tot, fill)
        nrecv = cnts[rank] if cnts else tot
        # where: "device" / "host" for both buffers, "dh" device sendbuf +
        # host recvbuf, "hd" the other way round (kinds mixed within a rank)
        sdev, rdev = where in ("device", "dh"), where in ("device", "hd")
        s = T.to_dev(S[rank]) if sdev else T.clone(S[rank]).view(np.uint8)
        if rdev:
            r = torch.zeros(max(nrecv, 1) * E, dtype=torch.uint8, device="cuda")
        else:
            r = np.zeros(max(nrecv, 1) * E, np.uint8)
        if coll == "ar":
            rc = mvx.MPI_Allreduce(s, r, tot, dtype, op, comm)
        elif coll == "red":
            rc = mvx.MPI_Reduce(s, r, tot, dtype, op, root, comm)
        elif coll == "scan":
            rc = mvx.MPI_Scan(s, r, tot, dtype, op, comm)
        else:
            rc = mvx.MPI_Reduce_scatter(s, r, cnts, dtype, op, comm)
        got = r if isinstance(r, np.ndarray) else T.from_dev(r)
        R0 = [np.zeros(max(cnts[q] if cnts else tot, 1), S[0].dtype) for q in range(world)]
        s8, r8 = [x.view(np.uint8) for x in S], [x.view(np.uint8) for x in R0]
        if coll == "ar":
            rref = O.allreduce(s8, r8, tot, dtype, op)
        elif coll == "red":
            rref = O.reduce(s8, r8, tot, dtype, op, root)
        elif coll == "scan":
            rref = O.scan(s8, r8, tot, dtype, op)
        else:
            rref = O.reduce_scatter(s8, r8, cnts, dtype, op)
        report["checked"] += 1
        # which exchange variant the call actually ran (mvx_comm_last_exchange)
        ran = report["ran"].setdefault(tag.split()[0] if tag else "-", {})
        key = str(comm.last_exchange())
        ran[key] = ran.get(key, 0) + 1
        ok = rc == rref[rank]
        # a 329 rank's recvbuf too: an undefined pair moves the data as the
        # reference's algorithm does
        if ok and rc in (0, 329) and (coll != "red" or rank == root) and nrecv > 0:
            try:
                T.assert_same(op, dtype, got[: nrecv * E], R0[rank][:nrecv], typemap_only=True)
            except AssertionError as e:
                ok = False
                tag += " " + str(e)[:200]
        if not ok:
            report["fails"].append([coll, dtype, op, tot, where, root, rc, rref[rank], tag])

    modes = [("p2p", mvx.EXCH_P2P, 0), ("pipe", mvx.EXCH_PIPE, 3), ("coll", mvx.EXCH_COLL, 0)]
    if suite == "small":
        cases = [(102, 10), (100, 10), (111, 17), (105, 8), (110, 18), (103, 6)]
        for name, mode, sl in modes:
            assert comm.set_exchange(mode, sl) == 0
            for op, dtype in cases:
                for where in ("device", "host"):
                    for n in (1, 10, 4097, 70001, 300000):
                        check("ar", dtype, op, n, where, tag=name)
                    for n in (5, 70001):
                        check("red", dtype, op, n, where, root=world - 1, tag=name)
                    for base in (3, 40000, 140000):
                        check("rs", dtype, op, [base + (q % 2) for q in range(world)], where, tag=name)
                        # equal blocks: the plans the COLL variant takes whole
                        check("rs", dtype, op, [base] * world, where, tag=name)
                    # a multiple of p above the Rabenseifner threshold (p = 4)
                    check("ar", dtype, op, 4096 * world * 4, where, tag=name)
                    check("scan", dtype, op, 5000, where, tag=name)
    elif suite == "random":
        # the same seeded case sequence on every rank (tests/test_gpu_fuzz.py's
        # draw, through the one-rank-per-process path)
        for i in range(int(os.environ.get("MVX_MP_CASES", "120"))):
            rng = np.random.default_rng(4242 + i)
            # MVX_MP_MODES=pipe: draw that variant only (same rng sequence)
            pool = [m for m in modes if m[0] in os.environ.get("MVX_MP_MODES", m[0]).split(",")]
            name, mode, sl = pool[int(rng.integers(0, len(modes))) % len(pool)]
            assert comm.set_exchange(mode, int(rng.integers(2, 6)) if mode == mvx.EXCH_PIPE else sl) == 0
            coll = str(rng.choice(["ar", "ar", "red", "rs", "scan"]))
            dtype = int(rng.choice(T.ALL_TYPES))
            op = int(rng.integers(100, 112))
            E = mvx.dtype_info(dtype)[0]
            n = int(rng.choice([1, 7, 255, 4097, 70001, 300007]))
            n = min(n, (16 << 20) // E // world)
            where = str(rng.choice(["device", "host", "dh", "hd"]))
            root = int(rng.integers(0, world))
            if coll == "rs":
                check(coll, dtype, op, [max(0, n // world + int(rng.integers(-2, 3))) for _ in range(world)], where,
                      tag=name + " #%d" % i)
            else:
                check(coll, dtype, op, n, where, root=root, tag=name + " #%d" % i)
    elif suite == "graph":
        # graphs on: each job three times on the same buffers -- eager,
        # captured, replayed -- through the blocking call (the null stream:
        # fork / join onto the communicator's stream) and the stream-ordered
        # one on a torch stream; every result checked against the oracle
        report["graph_states"] = {}
        import ctypes
        v = ctypes.c_int()
        ctypes.CDLL("libamdhip64.so.7").hipRuntimeGetVersion(ctypes.byref(v))
        report["hip_runtime"] = v.value          # the runtime this process runs on (torch's)
        side = torch.cuda.Stream()
        comm.set_graphs(True)
        only = os.environ.get("MVX_MP_MODES")       # e.g. "pipe": one variant only (diagnostics)
        for name, mode, sl in modes:
            if only and name not in only.split(","):
                continue
            assert comm.set_exchange(mode, sl) == 0
            for op, dtype in [(102, 10), (111, 17), (105, 8), (103, 6)]:
                for coll_kind, n in (("ar", 70001), ("ar", 4096 * world * 4), ("ar", 300000), ("rs", 140000),
                                     ("red", 70001)):
                    E = mvx.dtype_info(dtype)[0]
                    cnts = [n] * world if coll_kind == "rs" else None
                    tot = n * world if cnts else n
                    S = inputs(dtype, tot, None)
                    nrecv = n if cnts else tot
                    R0 = [np.zeros(max(cnts[q] if cnts else tot, 1), S[0].dtype) for q in range(world)]
                    s8, r8 = [x.view(np.uint8) for x in S], [x.view(np.uint8) for x in R0]
                    root = world - 1
                    if coll_kind == "ar":
                        rref = O.allreduce(s8, r8, tot, dtype, op)
                    elif coll_kind == "rs":
                        rref = O.reduce_scatter(s8, r8, cnts, dtype, op)
                    else:
                        rref = O.reduce(s8, r8, tot, dtype, op, root)
                    sbuf = T.to_dev(S[rank])
                    rbuf = torch.zeros(max(nrecv, 1) * E, dtype=torch.uint8, device="cuda")
                    for via in ("blocking", "stream"):
                        states = []
                        for rep in range(3):
                            if os.environ.get("MVX_MP_TRACE"):
                                sys.stderr.write("rank %d: %s %s op %d type %d n %d %s rep %d\n"
                                                 % (rank, name, coll_kind, op, dtype, n, via, rep))
                                sys.stderr.flush()
                            rbuf.zero_()
                            torch.cuda.synchronize()
                            if via == "blocking":
                                if coll_kind == "ar":
                                    rc = mvx.MPI_Allreduce(sbuf, rbuf, tot, dtype, op, comm)
                                elif coll_kind == "rs":
                                    rc = mvx.MPI_Reduce_scatter(sbuf, rbuf, cnts, dtype, op, comm)
                                else:
                                    rc = mvx.MPI_Reduce(sbuf, rbuf, tot, dtype, op, root, comm)
                            else:
                                side.wait_stream(torch.cuda.current_stream())
                                if coll_kind == "ar":
                                    rc = comm.allreduce_async(sbuf, rbuf, tot, dtype, op, side)
                                elif coll_kind == "rs":
                                    rc = comm.reduce_scatter_async(sbuf, rbuf, cnts, dtype, op, side)
                                else:
                                    rc = comm.reduce_async(sbuf, rbuf, tot, dtype, op, root, side)
                                side.synchronize()
                            states.append(comm.last_graph()[0])
                            report["checked"] += 1
                            ok = rc == rref[rank]
                            if ok and rc == 0 and (coll_kind != "red" or rank == root):
                                try:
                                    T.assert_same(op, dtype, T.from_dev(rbuf)[: nrecv * E], R0[rank][:nrecv],
                                                  typemap_only=True)
                                except AssertionError as e:
                                    ok = False
                                    report["fails"].append([coll_kind, dtype, op, tot, via, rep, str(e)[:200]])
                            elif not ok:
                                report["fails"].append([coll_kind, dtype, op, tot, via, rep, rc, rref[rank]])
                        key = "%s %s" % (name, via)
                        report["graph_states"].setdefault(key, []).append(states)
            report["graph_error"] = comm.last_graph()[1]
        report["graph_stats"] = comm.graph_stats()
        comm.set_graphs(False)
    elif suite == "mixed":
        # buffer kinds differing between the ranks of one call and between a
        # rank's two buffers (MPI allows both): rank r's kinds rotate through
        # host, device, device send + host recv, host send + device recv with
        # (case + r) -- host buffers run on HBM mirrors and move what a
        # device call moves, so the transfers pair up
        case = 0
        kinds = ("host", "device", "dh", "hd")
        for name, mode, sl in modes:
            assert comm.set_exchange(mode, sl) == 0
            for op, dtype in [(102, 10), (111, 17), (105, 8), (103, 6)]:
                for n in (10, 70001, 300000, 4096 * world * 4):
                    check("ar", dtype, op, n, kinds[(case + rank) % 4], tag=name)
                    case += 1
                for n in (5, 70001):
                    check("red", dtype, op, n, kinds[(case + rank) % 4], root=world - 1, tag=name)
                    case += 1
                for base in (3, 140000):
                    check("rs", dtype, op, [base] * world, kinds[(case + rank) % 4], tag=name)
                    case += 1
                check("scan", dtype, op, 5000, kinds[(case + rank) % 4], tag=name)
                case += 1
    elif suite == "sliced":
        # the slice schedule (mvx_stage.c: blocking calls at p > 1 from
        # MVX_SLICE_MIN_MIB on, every rank in the same slices whatever its
        # buffers' kind) at test sizes -- a 1 MiB threshold, 1 MiB slices --
        # with the kinds mixed between the ranks as in "mixed", and every
        # rank on host buffers, then every rank on device buffers
        os.environ["MVX_SLICE_MIN_MIB"] = "1"
        os.environ["MVX_SLICE_MIB"] = "1"
        case = 0
        for op, dtype in [(102, 10), (111, 17), (105, 8), (103, 6), (100, 11)]:
            E = mvx.dtype_info(dtype)[0]
            for how in ("mixed", "host", "device"):
                def where():
                    return how if how != "mixed" else ("host", "device", "dh", "hd")[(case + rank) % 4]
                for n in ((1 << 20) // E + 1, (3 << 20) // E + 7):
                    check("ar", dtype, op, n, where(), tag="sliced")
                    case += 1
                check("red", dtype, op, (5 << 20) // (2 * E) + 3, where(), root=world - 1, tag="sliced")
                case += 1
                base = (3 << 20) // E // world
                check("rs", dtype, op, [base + (q % 3) for q in range(world)], where(), tag="sliced")
                case += 1
                check("scan", dtype, op, (2 << 20) // E + 5, where(), tag="sliced")
                case += 1
        # agreed kinds (mvx_comm_set_call_kinds, what the MVAPICH shim passes):
        # every rank device -> the unsliced device path and its exchange
        # variant (PIPE here, reported as such); every rank host -> the
        # sliced pipeline.  A hint rank 0's buffers contradict: every rank
        # still runs the schedule the hint names (rank 0's host buffers
        # through HBM mirrors under DEVICE, its device buffers in place under
        # HOST), so the transfers pair and the bits are the oracle's
        assert comm.set_exchange(mvx.EXCH_PIPE, 3) == 0
        for op, dtype in [(102, 10), (111, 17)]:
            E = mvx.dtype_info(dtype)[0]
            n = (3 << 20) // E + 7
            for where, kinds in (("device", mvx.KINDS_DEVICE), ("host", mvx.KINDS_HOST)):
                assert comm.set_call_kinds(kinds) == 0
                check("ar", dtype, op, n, where, tag="agreed")
                report.setdefault("agreed_ran", []).append([where, comm.last_exchange()])
            for kinds, odd, usual in ((mvx.KINDS_DEVICE, "host", "device"), (mvx.KINDS_HOST, "device", "host")):
                assert comm.set_call_kinds(kinds) == 0
                check("ar", dtype, op, n, odd if rank == 0 else usual, tag="contradicted")
                report.setdefault("contradicted", []).append(comm.last_exchange())
        assert comm.set_exchange(mvx.EXCH_P2P, 0) == 0
        del os.environ["MVX_SLICE_MIN_MIB"], os.environ["MVX_SLICE_MIB"]
    else:
        # the BASELINE multi-GPU shapes at full size: C3, C4 (p = 4 in the
        # config; any p here), C5
        for name, mode, sl in modes:
            assert comm.set_exchange(mode, sl) == 0
            check("ar", 10, 102, 64 << 20, "device", tag=name + " c3", fill=0)
            check("rs", 8, 105, [(1 << 27) // world] * world, "device", tag=name + " c4", fill=2)
            check("ar", 17, 111, 64 << 20, "device", tag=name + " c5", fill=4)
            torch.cuda.empty_cache()
    if transport == "host":
        report["transport_errors"] = comm.transport.errors
    comm.free()
    dist.barrier()
    dist.destroy_process_group()
    with open(out, "w") as f:
        json.dump(report, f)


if __name__ == "__main__":
    main()
