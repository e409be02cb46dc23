#!/usr/bin/env python3
"""Per-config combine-kernel throughput on one MI355X (HBM roofline).

For each BASELINE config the device arithmetic is one k-leaf combine over the
rank's block.  This times exactly that kernel, with the
shapes the multi-GPU run gives each rank, on rotating buffer sets so that no
operand is served from the 256 MiB Infinity Cache:

  C2  apply  k=2  SUM   f32         256 MiB vectors        (bench.py's N=1)
  C3  tree   k=8  SUM   f32         8 x 32 MiB -> 32 MiB   (Allreduce 256 MiB, p=8)
  C4  chain  k=4  BAND  int64       4 x 256 MiB -> 256 MiB (Reduce_scatter 1 GiB, p=4)
  C5  tree   k=8  MAXLOC FLOAT_INT  8 x 64 MiB -> 64 MiB   (Allreduce 512 MiB, p=8)

Prints one JSON line per config: algorithmic bytes, kernel time (HIP events on
the launch stream), GB/s and fraction of the 8 TB/s HBM peak.
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MIB = 1 << 20
PEAK = 8000.0


def run(mvx, name, op, dtype, k, shape, leaf_bytes, sets, reps=20, warm=3, quiet=False):
    import torch
    n_elems = leaf_bytes // mvx.dtype_info(dtype)[0]
    bufs = []
    for s in range(sets):
        if k > 2:
            # the executor's staging pool: shard slots back to back, 4 KiB
            # staggered (mvx_exec.c exec_layout)
            big = torch.randint(0, 1 << 30, (k * (leaf_bytes + 4096) // 4,), dtype=torch.int32, device="cuda")
            leaves = [big[q * (leaf_bytes + 4096) // 4:][: leaf_bytes // 4] for q in range(k)]
        else:
            leaves = [torch.randint(0, 1 << 30, (leaf_bytes // 4,), dtype=torch.int32, device="cuda")
                      for _ in range(k)]
        if os.environ.get("BK_CONST"):      # every word 0x3c3c3c3c (does the data pattern matter?)
            for x in leaves:
                x.fill_(0x3c3c3c3c)
        elif dtype == mvx.MPI_FLOAT:        # in place: keeps the slot layout
            leaves = [x.view(torch.float32).copy_(x.float() * 1e-6) for x in leaves]
        elif dtype in (mvx.MPI_LONG_DOUBLE, mvx.MPI_LONG_DOUBLE_INT):
            leaves = [_x87_values(x, dtype, mvx) for x in leaves]
        dst = torch.empty(leaf_bytes // 4, dtype=torch.int32, device="cuda")
        bufs.append((leaves, dst))
    stream = torch.cuda.current_stream()

    def launch(i):
        leaves, dst = bufs[i % sets]
        if k == 2 and shape == 1:
            rc = mvx.op_apply(op, dtype, leaves[1], leaves[0], n_elems, stream)
        else:
            rc = mvx.op_combine(op, dtype, leaves, dst, n_elems, shape=shape, stream=stream)
        assert rc == 0, rc

    for i in range(warm):
        launch(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(reps):
        launch(i)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    alg = (k + 1) * leaf_bytes
    gbs = alg / (us * 1e-6) / 1e9
    out = {"config": name, "kernel": mvx.last_kernel(), "k": k, "leaf_bytes": leaf_bytes,
           "alg_bytes_per_launch": alg, "kernel_us": round(us, 2), "achieved_GBps": round(gbs, 1),
           "hbm_frac": round(gbs / PEAK, 4), "sets": sets}
    if not quiet:
        print(json.dumps(out), flush=True)
    del bufs
    torch.cuda.empty_cache()
    return out


def _x87_values(x, dtype, mvx):
    """Finite x87 values near 1 (normal operands: the emulation's main path)."""
    import torch
    w = x.view(torch.int64).view(-1, 2 if dtype == mvx.MPI_LONG_DOUBLE else 4)
    w[:, 0] |= torch.iinfo(torch.int64).min                       # integer bit
    w[:, 1] = 16383 + (w[:, 1] & 15) - 8 + ((w[:, 1] >> 8) & 1) * 0x8000
    return x


def main():
    mvx = importlib.import_module("mvapich-cce_amd")
    run(mvx, "C2", mvx.MPI_SUM, mvx.MPI_FLOAT, 2, 1, 256 * MIB, 4)
    run(mvx, "C3", mvx.MPI_SUM, mvx.MPI_FLOAT, 8, 0, 32 * MIB, 4)
    run(mvx, "C4", mvx.MPI_BAND, mvx.MPI_LONG, 4, 1, 256 * MIB, 2)
    run(mvx, "C5", mvx.MPI_MAXLOC, mvx.MPI_FLOAT_INT, 8, 0, 64 * MIB, 2)
    if "sweep" in sys.argv[1:]:
        # edge effects vs steady state: the same programs at other sizes, and
        # the plain op at the C3 / C5 launch sizes
        for mib in (32, 96, 512):
            run(mvx, "C2-%dMiB" % mib, mvx.MPI_SUM, mvx.MPI_FLOAT, 2, 1, mib * MIB, 4 if mib < 512 else 2)
        for mib in (16, 64, 128, 256):
            run(mvx, "C3-leaf%dMiB" % mib, mvx.MPI_SUM, mvx.MPI_FLOAT, 8, 0, mib * MIB, 4 if mib <= 64 else 2)
        for mib in (32, 128, 256):
            run(mvx, "C5-leaf%dMiB" % mib, mvx.MPI_MAXLOC, mvx.MPI_FLOAT_INT, 8, 0, mib * MIB, 4 if mib <= 64 else 2)
    if "all" in sys.argv[1:] and "all-tree" not in sys.argv[1:]:
        # every defined (op, type) pair's apply kernel at 256 MiB vectors
        # (the op functions' and a 2-leaf combine's kernel): the whole op
        # table against the HBM peak, one line each
        hip = mvx.hip()
        types = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 17, 18, 19, 20, 21, 22, 23, 24,
                 25, 26, 27, 28, 29, 30, 31, 32, 33]
        for op in range(100, 112):
            for t in types:
                if hip.mvx_op_supported(op, t) != 1:
                    continue
                run(mvx, "A-%d-%d" % (op, t), op, t, 2, 1, 256 * MIB, 4, reps=10, warm=2)
    if "all-tree" in sys.argv[1:]:
        # the same pairs as 8-leaf trees over 32 MiB leaves (the C3 shape)
        hip = mvx.hip()
        types = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 17, 18, 19, 20, 21, 22, 23, 24,
                 25, 26, 27, 28, 29, 30, 31, 32, 33]
        for op in range(100, 112):
            for t in types:
                if hip.mvx_op_supported(op, t) != 1:
                    continue
                run(mvx, "T-%d-%d" % (op, t), op, t, 8, 0, 32 * MIB, 4, reps=10, warm=2)
    if "ks" in sys.argv[1:]:
        # every leaf count 2..8, tree and chain (the masked program where no
        # body kernel fits: k = 3, 5, 6, 7), f32 SUM and int64 BAND, 32 MiB leaves
        for op, t in ((mvx.MPI_SUM, mvx.MPI_FLOAT), (mvx.MPI_BAND, mvx.MPI_LONG)):
            for shape in (0, 1):
                for k in range(2, 9):
                    run(mvx, "K-%d-%d-%s-k%d" % (op, t, "tree" if shape == 0 else "chain", k), op, t, k, shape,
                        32 * MIB, 4, reps=10, warm=2)
    if "x87" in sys.argv[1:]:
        # x87 long double (integer emulation): apply and the C3 / C5 shapes
        run(mvx, "X2-sum", mvx.MPI_SUM, mvx.MPI_LONG_DOUBLE, 2, 1, 256 * MIB, 4)
        run(mvx, "X2-prod", mvx.MPI_PROD, mvx.MPI_LONG_DOUBLE, 2, 1, 256 * MIB, 4)
        run(mvx, "X2-max", mvx.MPI_MAX, mvx.MPI_LONG_DOUBLE, 2, 1, 256 * MIB, 4)
        run(mvx, "X3-sum", mvx.MPI_SUM, mvx.MPI_LONG_DOUBLE, 8, 0, 32 * MIB, 4)
        run(mvx, "X5-maxloc", mvx.MPI_MAXLOC, mvx.MPI_LONG_DOUBLE_INT, 8, 0, 64 * MIB, 2)
        run(mvx, "X5-minloc", mvx.MPI_MINLOC, mvx.MPI_LONG_DOUBLE_INT, 8, 0, 64 * MIB, 2)
        run(mvx, "X3-max", mvx.MPI_MAX, mvx.MPI_LONG_DOUBLE, 8, 0, 32 * MIB, 4)


if __name__ == "__main__":
    main()
