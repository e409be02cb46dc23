#!/usr/bin/env python3
"""Benchmark of the MI355X MPI reduction path (BASELINE.json metric).

  N = 1  config 2: device-resident pairwise MPI_SUM on MPI_FLOAT, 256 MiB
         vectors -- one step = one local MPI_Op kernel (inout = in + inout).
  N > 1  config 3 shape: MPI_Allreduce(MPI_SUM, MPI_FLOAT) of 256 MiB per
         rank, one process per GPU (torchrun), RCCL over xGMI for the
         exchanges + the reference-order combine kernel.

value = bytes of input vectors reduced per second over the whole job
(N x 256 MiB per step / step time), GiB/s.  Inputs are resident in HBM before
the timed region.  See DESIGN.md section 6 for the roofline accounting.
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MIB = 1 << 20
GIB = 1 << 30
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, chip-level parameters
XGMI_LINK_GBS = 153.0           # BASELINE.md section 3 (per link, per direction)
MPI_SUM, MPI_FLOAT = 102, 10


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mib", type=int, default=256, help="vector size per rank (MiB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r01", "pmc_c2.json"),
                    help="committed rocprofv3 PMC summary for the traffic field")
    ap.add_argument("--block-cap", type=int, default=0)
    ap.add_argument("--nt-min-log2", type=int, default=0, help="-1 disables non-temporal loads/stores")
    ap.add_argument("--sets", type=int, default=4,
                    help="input sets used round-robin (4 x 512 MiB keeps every step out of the 256 MiB "
                         "Infinity Cache: the number is HBM-bound, not cache-bound)")
    return ap.parse_args()


def synth(n, rank, device):
    """Mixed-sign f32 with an exponent spread, made on the GPU."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(0x9E3779B9 ^ (rank * 1000003 + 1))
    m = torch.randint(-1000000, 1000001, (n,), generator=g, device=device, dtype=torch.int32)
    s = torch.randint(1, 1001, (n,), generator=g, device=device, dtype=torch.int32)
    return (m.to(torch.float32) * 1e-3 * s.to(torch.float32)).contiguous()


def cpu_baseline(n_bytes, seconds):
    """Oracle MPIR_SUM (oracle/cpu_ops.c, the reference's loop) on 1 host core."""
    import numpy as np
    from oracle import oracle as O
    n = n_bytes // 4
    a = np.empty(n, np.float32)
    b = np.empty(n, np.float32)
    O.fill(a, n, 0, 0)
    O.fill(b, n, 0, 1)
    O.op(MPI_SUM, MPI_FLOAT, a.view(np.uint8), b.view(np.uint8), n)  # warm pages
    reps, t0 = 0, time.perf_counter()
    while True:
        O.op(MPI_SUM, MPI_FLOAT, a.view(np.uint8), b.view(np.uint8), n)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"value": round(n_bytes * reps / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": "oracle MPIR_SUM float32, %d MiB vectors x %d reps (%.1f s) on 1 host core"
                      % (n_bytes // MIB, reps, dt),
            "cpu": _cpu_model()}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(path, kernel, nbytes):
    """Per-launch HBM bytes from a committed rocprofv3 PMC summary, if it was
    collected for this kernel at this size (FETCH_SIZE doubled on gfx950)."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("kernel_tag") != kernel or d.get("vector_bytes") != nbytes:
        return None
    return d.get("hbm_bytes_per_launch")


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    mvx = importlib.import_module("mvapich-cce_amd")
    if args.block_cap or args.nt_min_log2:
        mvx.set_launch(args.block_cap, args.nt_min_log2)

    nbytes = args.mib * MIB
    n = nbytes // 4
    stream = torch.cuda.current_stream()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    it = [0]
    if world == 1:
        x_in = [synth(n, 2 * s, dev) for s in range(args.sets)]
        x_io = [synth(n, 2 * s + 1, dev) for s in range(args.sets)]

        def step():
            s = it[0] % args.sets
            it[0] += 1
            rc = mvx.op_apply(MPI_SUM, MPI_FLOAT, x_in[s], x_io[s], n, stream)
            if rc:
                raise RuntimeError("mvx_op_apply rc=%d" % rc)
        comm = None
    else:
        comm = mvx.Comm.from_torch_distributed(local)
        sets = max(1, min(args.sets, 2))
        sendbuf = [synth(n, rank * 16 + s, dev) for s in range(sets)]
        recvbuf = [torch.empty_like(sendbuf[0]) for _ in range(sets)]
        comm.reserve(2 * nbytes)

        def step():
            s = it[0] % sets
            it[0] += 1
            rc = comm.allreduce_async(sendbuf[s], recvbuf[s], n, MPI_FLOAT, MPI_SUM, stream)
            if rc:
                raise RuntimeError("mvx_allreduce_async rc=%d" % rc)

    for _ in range(args.warmup):
        step()
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1)
    t_local = max(wall, dev_ms / 1e3)
    if world > 1:
        t = torch.tensor([t_local], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_job = float(t.item())
    else:
        t_job = t_local
    kernel = mvx.last_kernel()
    ms_per_step = t_job * 1e3 / args.steps
    value = world * nbytes * args.steps / t_job / GIB

    if world == 1:
        kern_s = dev_ms / 1e3 / args.steps           # HIP events on the launch stream
        alg_bytes = 3 * nbytes                         # read in, read inout, write inout
        achieved = alg_bytes / kern_s / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(args.pmc, kernel, nbytes),
                "kernel": kernel, "kernel_us": round(kern_s * 1e6, 2), "alg_bytes_per_launch": alg_bytes}
        workload = ("config2: device-resident pairwise MPI_SUM float32 %d MiB (local MPI_Op kernel), "
                    "%d input sets round-robin" % (args.mib, args.sets))
        par = "single GPU"
    else:
        p = world
        busbw = 2 * (p - 1) / p * nbytes / (ms_per_step / 1e3) / 1e9
        links = min(p - 1, 7)
        peak = links * XGMI_LINK_GBS
        roof = {"bound": "xgmi", "achieved": round(busbw, 1), "peak": peak, "unit": "GB/s",
                "frac": round(busbw / peak, 4), "traffic": None, "kernel": kernel,
                "note": "busbw = 2(p-1)/p*S/t against %d direct xGMI links" % links}
        workload = "config3-shape: MPI_Allreduce SUM float32 %d MiB per rank, RCCL xGMI exchange + combine" % args.mib
        par = "dp%d (blocks sharded over ranks)" % p

    out = {
        "metric": "GiB/s device-resident Allreduce(SUM,float32) at 1/2/4/8 GPUs; % HBM/xGMI peak",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (mixed-sign f32, generated on device)",
        "config": {"workload": workload, "vector_bytes_per_rank": nbytes, "op": "MPI_SUM",
                   "datatype": "MPI_FLOAT", "parallelism": par},
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(nbytes, args.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    if comm is not None:
        comm.free()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
