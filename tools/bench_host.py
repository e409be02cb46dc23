#!/usr/bin/env python3
"""Latency / throughput of the blocking calls when MPI user buffers live in
host memory, against the same calls on device buffers.

The reference's buffers are host memory; on MI355X every byte then crosses
PCIe (H2D in, D2H out).  For float32 vectors of 8 B ... 256 MiB, one line per
(case, size) with the median call time and the rate per vector:

  op_device     MPIR_SUM(invec, inoutvec), both operands in HBM
  op_pageable   the same on malloc'd (pageable) numpy arrays (2 H2D + 1 D2H)
  op_pinned     the same on pinned host tensors
  ar1_device    MPI_Allreduce(SUM) at p = 1 over RCCL, device buffers
  ar1_pageable  the same on pageable host buffers (staged pipeline: H2D,
                device collective, D2H)
  ar1_pinned    the same on pinned host buffers (DMA straight from them)
  ar4_local_*   a 4-rank virtual communicator (one process, loopback), the
                sum of 4 vectors: host buffers staged per rank
  *_registered  pageable numpy arrays with the registration cache on
                (mvx_host_register_enable): the first call page-locks them
                ("first_us"), the timed calls DMA them directly

Every result is checked against numpy (float32 sums of small integers are
exact).  usage: bench_host.py [--min-mib M] [--max-mib 256] [--cases a,b,...]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MIB, GIB = 1 << 20, 1 << 30
ALL = ["op_device", "op_pageable", "op_pinned", "op_registered", "ar1_device", "ar1_pageable", "ar1_pinned",
       "ar1_registered", "ar4_local_device", "ar4_local_pageable"]


def timeit(fn, budget=0.25, max_reps=2000, warm=True):
    """median seconds of fn over as many calls as fit in `budget` (>= 3)"""
    if warm:
        fn()
    ts = []
    t_end = time.perf_counter() + budget
    while len(ts) < 3 or (time.perf_counter() < t_end and len(ts) < max_reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], len(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=256)
    ap.add_argument("--min-mib", type=int, default=0, help="start the size sweep here (default 8 bytes)")
    ap.add_argument("--cases", default=",".join(ALL))
    args = ap.parse_args()
    cases = args.cases.split(",")

    import numpy as np
    import torch
    import torch.distributed as dist
    mvx = importlib.import_module("mvapich-cce_amd")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29544")
    dist.init_process_group("gloo", rank=0, world_size=1)
    comm = mvx.Comm.from_torch_distributed(0)
    local = mvx.Comm.local_ranks(4, 0)
    F, SUM = mvx.MPI_FLOAT, mvx.MPI_SUM

    sizes = []
    b = args.min_mib * MIB if args.min_mib else 8
    while b <= args.max_mib * MIB:
        sizes.append(b)
        b *= 4
    if sizes[-1] != args.max_mib * MIB:
        sizes.append(args.max_mib * MIB)

    rng = np.random.default_rng(0)
    for nbytes in sizes:
        n = nbytes // 4
        a = rng.integers(-8, 8, n).astype(np.float32)
        b0 = rng.integers(-8, 8, n).astype(np.float32)
        want = a + b0
        for case in cases:
            first = None
            mvx.host_register_enable(case.endswith("_registered"))
            if case.startswith("op_"):
                where = case[3:]
                if where == "device":
                    x, y = torch.from_numpy(a).cuda(), torch.from_numpy(b0).cuda()
                elif where == "pinned":
                    x, y = torch.from_numpy(a).pin_memory(), torch.from_numpy(b0).pin_memory()
                else:
                    x, y = a.copy(), b0.copy()
                y0 = y.clone() if torch.is_tensor(y) else y.copy()

                def call():
                    y.copy_(y0) if torch.is_tensor(y) else np.copyto(y, y0)
                    mvx.MPIR_call("MPIR_SUM", x, y, n, F)

                t0 = time.perf_counter()
                call()
                first = time.perf_counter() - t0
                got = y.cpu().numpy() if torch.is_tensor(y) else y
                assert mvx.op_errno() == 0 and np.array_equal(got, want), case

                def fn():
                    mvx.MPIR_call("MPIR_SUM", x, y, n, F)
                t, reps = timeit(fn)
                pcie = {"device": 0, "pinned": 3, "pageable": 3, "registered": 3}[where] * nbytes
            elif case.startswith("ar1_"):
                where = case[4:]
                if where == "device":
                    x, y = torch.from_numpy(a).cuda(), torch.zeros(n, dtype=torch.float32, device="cuda")
                elif where == "pinned":
                    x, y = torch.from_numpy(a).pin_memory(), torch.zeros(n, dtype=torch.float32).pin_memory()
                else:
                    x, y = a.copy(), np.zeros(n, np.float32)

                def fn():
                    assert mvx.MPI_Allreduce(x, y, n, F, SUM, comm) == 0
                t0 = time.perf_counter()
                fn()
                first = time.perf_counter() - t0
                got = y.cpu().numpy() if torch.is_tensor(y) else y
                assert np.array_equal(got, a), case
                t, reps = timeit(fn)
                pcie = 0 if where == "device" else 2 * nbytes
            else:
                where = case[len("ar4_local_"):]
                S = [a, b0, a, b0]
                if where == "device":
                    xs = [torch.from_numpy(s).cuda() for s in S]
                    ys = [torch.zeros(n, dtype=torch.float32, device="cuda") for _ in S]
                else:
                    xs = [s.copy() for s in S]
                    ys = [np.zeros(n, np.float32) for _ in S]

                def fn():
                    r, rcs = local.allreduce_multi(xs, ys, n, F, SUM)
                    torch.cuda.synchronize()      # the *_multi calls are stream-ordered on device buffers
                    assert r == 0 and rcs == [0] * 4
                fn()
                for yy in ys:
                    got = yy.cpu().numpy() if torch.is_tensor(yy) else yy
                    assert np.array_equal(got, 2 * want), case
                t, reps = timeit(fn)
                pcie = 0 if where == "device" else 8 * nbytes
                del xs, ys
            reg = mvx.host_register_stats()
            mvx.host_register_enable(False)          # drops every registration
            print(json.dumps({"case": case, "bytes": nbytes, "us": round(t * 1e6, 2), "reps": reps,
                              "first_us": round(first * 1e6, 2) if first is not None else None,
                              "registered": reg if case.endswith("_registered") else None,
                              "GiB_per_s_per_vector": round(nbytes / t / GIB, 3),
                              "pcie_bytes": pcie, "pcie_GBps": round(pcie / t / 1e9, 2) if pcie else None}),
                  flush=True)
        torch.cuda.empty_cache()
    local.free()
    comm.free()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
