#!/usr/bin/env python3
"""End-to-end rate when MPI user buffers live in host memory.

The reference's buffers are host memory; on MI355X every byte then crosses
PCIe (H2D in, D2H out).  Times, per 256 MiB float32 vector:

  op_pageable   MPIR_SUM(invec, inoutvec) on malloc'd (pageable) numpy arrays
  op_pinned     the same on pinned host tensors
  op_device     the same with both operands already in HBM (the device rate)
  ar1_pageable  MPI_Allreduce(SUM) at p = 1 on pageable host buffers (H2D,
                device collective, D2H)
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MIB, GIB = 1 << 20, 1 << 30


def timeit(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    import numpy as np
    import torch
    mvx = importlib.import_module("mvapich-cce_amd")
    nbytes = 256 * MIB
    n = nbytes // 4
    a = np.random.default_rng(0).standard_normal(n).astype(np.float32)
    b = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    res = {}

    def op(x, y):
        mvx.MPIR_call("MPIR_SUM", x, y, n, mvx.MPI_FLOAT)
        assert mvx.op_errno() == 0
    t = timeit(lambda: op(a, b))
    res["op_pageable"] = t
    pa, pb = torch.from_numpy(a).pin_memory(), torch.from_numpy(b).pin_memory()
    res["op_pinned"] = timeit(lambda: op(pa, pb))
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    res["op_device"] = timeit(lambda: op(da, db))

    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29544")
    dist.init_process_group("gloo", rank=0, world_size=1)
    comm = mvx.Comm.from_torch_distributed(0)
    r = np.empty_like(a)
    res["ar1_pageable"] = timeit(lambda: mvx.MPI_Allreduce(a, r, n, mvx.MPI_FLOAT, mvx.MPI_SUM, comm))
    comm.free()
    for k, v in res.items():
        pcie = {"op_pageable": 3, "op_pinned": 3, "op_device": 0, "ar1_pageable": 2}[k] * nbytes
        print(json.dumps({"case": k, "vector_MiB": 256, "ms": round(v * 1e3, 3),
                          "GiB_per_s_per_vector": round(nbytes / v / GIB, 2),
                          "pcie_bytes": pcie, "pcie_GBps": round(pcie / v / 1e9, 1) if pcie else None}))


if __name__ == "__main__":
    main()
