#!/usr/bin/env python3
"""CPU baseline of the collective configs.

The reference's own schedules (intra_fns_new.c: binomial Reduce, Rabenseifner
Allreduce, pairwise Reduce_scatter) restated in oracle/cpu_coll.c and run by
p host threads -- one core per rank, shared memory as the ch_shmem device's
medium -- on the BASELINE configs' inputs:

  C1  MPI_Reduce  SUM  MPI_INT        1 MiB per rank, p = 2, root 0
  C3  MPI_Allreduce SUM MPI_FLOAT     256 MiB per rank, p = 8
  C4  MPI_Reduce_scatter BAND MPI_LONG 1 GiB per rank, p = 4
  C5  MPI_Allreduce MAXLOC MPI_FLOAT_INT 64 Mi pairs per rank, p = 8

One JSON line per config: seconds per collective (best and mean over the
timed reps) and GiB/s of per-rank payload.  A reported baseline (kind
"port": the oracle's restatement, not the reference binary), not a target.
Pass a scale < 1 to shrink C3-C5 (e.g. 0.25) where host memory is short.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

MIB, GIB = 1 << 20, 1 << 30


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def run(name, coll, p, n, dtype, op, dist, budget_s=6.0, recvcnts=None, int_ramp=False):
    e, _ = O.dtype_info(dtype)
    sends = []
    for r in range(p):
        a = np.empty(n * e, np.uint8)
        if int_ramp:                                  # C1: a[i] = i * (rank + 1)
            a.view(np.int32)[:] = np.arange(n, dtype=np.int32) * (r + 1)
        else:
            O.fill(a, n, dist, r)
        sends.append(a)
    if coll == 3:
        recvs = [np.zeros(c * e, np.uint8) for c in recvcnts]
        tmps = [np.zeros(c * e + 64, np.uint8) for c in recvcnts]   # pairwise: one block
    else:
        recvs = [np.zeros(n * e, np.uint8) for _ in range(p)]
        tmps = [np.zeros(n * e + 64, np.uint8) for _ in range(p)]
    t1 = O.threads_coll(coll, sends, recvs, tmps, n, dtype, op, recvcnts=recvcnts, reps=1)   # warm pages
    reps = max(1, min(200, int(budget_s / max(t1, 1e-6))))
    best, t0 = float("inf"), time.perf_counter()
    done = 0
    while done < reps:
        t = O.threads_coll(coll, sends, recvs, tmps, n, dtype, op, recvcnts=recvcnts, reps=1)
        best = min(best, t)
        done += 1
    mean = (time.perf_counter() - t0) / done
    payload = (sum(recvcnts) if coll == 3 else n) * e
    out = {"config": name, "p": p, "cores": p, "kind": "port", "reps": done,
           "best_ms": round(best * 1e3, 3), "mean_ms": round(mean * 1e3, 3),
           "GiB_per_s_per_rank": round(payload / best / GIB, 3),
           "bytes_per_rank": payload, "cpu": cpu_model(), "nproc": os.cpu_count()}
    print(json.dumps(out), flush=True)
    return out


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    run("C1 Reduce SUM INT 1MiB", 2, 2, 262144, 6, 102, 0, budget_s=2.0, int_ramp=True)
    n3 = int((64 << 20) * scale)
    run("C3 Allreduce SUM FLOAT 256MiB", 1, 8, n3, 10, 102, 0)
    n4 = int((1 << 27) * scale)
    run("C4 Reduce_scatter BAND LONG 1GiB", 3, 4, n4, 8, 105, 2, recvcnts=[n4 // 4] * 4)
    n5 = int((64 << 20) * scale)
    run("C5 Allreduce MAXLOC FLOAT_INT 64Mi", 1, 8, n5, 17, 111, 4)


if __name__ == "__main__":
    main()
