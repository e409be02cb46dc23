#!/usr/bin/env python3
"""Host-buffer MPI_Allreduce(SUM, float32) at p > 1: the end-to-end rate of a
rank whose buffers are host memory (PCIe-inclusive),
with its peers on host or device buffers.  One process per rank, started by
the caller with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun, or
tools/prof_host_multi.sh under rocprofv3 for the copy / kernel overlap).

  python3 tools/host_multi.py --mib 256 --kinds host,device --reps 5 \
      [--transport rccl-net|rccl] [--pinned]

Every rank checks its result bit-exact against the oracle's replay of the
reference schedule on the first call.  Prints one JSON line per rank:
ms per call (median of --reps after one warm call), GB/s of the vector, the
schedule the call took (MVX_SLICE_MIN_MIB: sliced vs HBM mirrors).
"""
import argparse
import importlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--kinds", default="host,device", help="buffer kind per rank, cycled")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--transport", default="rccl-net", choices=["rccl-net", "rccl"])
    ap.add_argument("--pinned", action="store_true", help="page-locked host buffers (torch pin_memory)")
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if a.transport == "rccl-net":
        importlib.import_module("mvapich-cce_amd.transport").rccl_net_env(rank)
    import numpy as np
    import torch
    import torch.distributed as dist

    mvx = importlib.import_module("mvapich-cce_amd")
    dev = rank % torch.cuda.device_count() if a.transport == "rccl-net" else rank
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = mvx.Comm.from_torch_distributed(dev)
    kinds = a.kinds.split(",")
    kind = kinds[rank % len(kinds)]
    n = a.mib * (1 << 20) // 4
    rng = np.random.default_rng(1234 + rank)
    x = rng.integers(-64, 64, n).astype(np.float32)      # small integers: every order gives the same sum
    if kind == "device":
        s = torch.from_numpy(x).cuda()
        r = torch.zeros(n, dtype=torch.float32, device="cuda")
    elif a.pinned:
        s = torch.from_numpy(x).pin_memory()
        r = torch.zeros(n, dtype=torch.float32).pin_memory()
    else:
        s, r = x, np.zeros(n, np.float32)
    ok = None
    times = []
    for rep in range(a.reps + 1):
        dist.barrier()
        t0 = time.perf_counter()
        rc = mvx.MPI_Allreduce(s, r, n, mvx.MPI_FLOAT, mvx.MPI_SUM, comm)
        if kind == "device":
            torch.cuda.synchronize()
        t = time.perf_counter() - t0
        assert rc == 0, rc
        if rep == 0:
            if not a.no_check:
                xs = [np.random.default_rng(1234 + q).integers(-64, 64, n).astype(np.float32) for q in range(world)]
                got = r.cpu().numpy() if torch.is_tensor(r) else r
                ok = bool(np.array_equal(got, np.sum(xs, axis=0, dtype=np.float32)))
        else:
            times.append(t)
    ms = statistics.median(times) * 1e3
    slice_min = int(os.environ.get("MVX_SLICE_MIN_MIB", "64"))
    print(json.dumps({"rank": rank, "world": world, "kind": kind + (" pinned" if a.pinned and kind == "host" else ""),
                      "kinds": kinds, "mib": a.mib, "ms": round(ms, 3), "ms_all": [round(t * 1e3, 3) for t in times],
                      "GBs": round(n * 4 / (ms * 1e-3) / 1e9, 2), "parity": ok,
                      "schedule": "sliced" if a.mib >= slice_min else "unsliced",
                      "slice_mib": int(os.environ.get("MVX_SLICE_MIB", "32")), "transport": a.transport,
                      "exchange_ran": {-1: "none", 0: "p2p", 1: "pipe", 2: "coll"}.get(comm.last_exchange())}),
          flush=True)
    comm.free()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
