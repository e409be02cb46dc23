#!/usr/bin/env python3
"""Pack / unpack kernel rates for derived datatypes with holes (the types
that move packed): mvx_type_pack (extent layout ->
type-map bytes) and mvx_type_unpack (back, writing type-map bytes only) on
one MI355X, HIP events on the launch stream, two rotating buffer sets of a
~256 MiB extent span each (so the Infinity Cache serves neither).

One JSON line per (type, direction): packed bytes per launch, time, the
rate of the type-map bytes moved both ways (read + write of `size` bytes per
element: the algorithmic bytes), and the rate counting every 128-byte line
of the extent span the type map touches (what HBM must move at least)
against the 8 TB/s peak.

  python3 tools/bench_pack.py
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PEAK = 8000.0
SPAN = 256 << 20


def lines_touched(blocks, ext, n):
    """128-byte lines of n elements' extent span that the type map touches:
    one element's (offset, length) blocks tiled every `ext` bytes over a
    whole number of lines, scaled to n elements"""
    import numpy as np
    reps = 128 // int(np.gcd(ext, 128))
    mask = np.zeros(ext * reps + 256, bool)
    for r in range(reps):
        for o, ln in blocks:
            mask[r * ext + o:r * ext + o + ln] = True
    used = mask[: (len(mask) // 128) * 128].reshape(-1, 128).any(axis=1).sum()
    return int(used) * 128 * n / reps


def main():
    import torch
    mvx = importlib.import_module("mvapich-cce_amd")
    F, D, I = mvx.MPI_FLOAT, mvx.MPI_DOUBLE, mvx.MPI_INT
    def vec(count, bl, stride, e):      # (offset, length) blocks of one vector element
        return [(i * stride * e, bl * e) for i in range(count)]
    cases = [
        ("vector(2,1,2,FLOAT) every other float", mvx.MPI_Type_vector, (2, 1, 2, F), vec(2, 1, 2, 4)),
        ("vector(8,1,4,DOUBLE) 8 B of every 32", mvx.MPI_Type_vector, (8, 1, 4, D), vec(8, 1, 4, 8)),
        ("vector(64,16,32,FLOAT) 64 B of every 128", mvx.MPI_Type_vector, (64, 16, 32, F), vec(64, 16, 32, 4)),
        ("vector(16,64,128,FLOAT) 256 B of every 512", mvx.MPI_Type_vector, (16, 64, 128, F), vec(16, 64, 128, 4)),
        ("vector(4,1000,1024,FLOAT) 4000 B of every 4096", mvx.MPI_Type_vector, (4, 1000, 1024, F),
         vec(4, 1000, 1024, 4)),
        ("struct{int; hole; double} 12 B of 16", mvx.MPI_Type_struct, (2, [1, 1], [0, 8], [I, D]), [(0, 4), (8, 8)]),
        ("vector(2,1,2,CHAR) every other byte", mvx.MPI_Type_vector, (2, 1, 2, mvx.MPI_CHAR), vec(2, 1, 2, 1)),
        ("struct{char; hole; int} 5 B of 8", mvx.MPI_Type_struct, (2, [1, 1], [0, 4], [mvx.MPI_CHAR, I]),
         [(0, 1), (4, 4)]),
        ("vector(4,1,2,SHORT) every other short", mvx.MPI_Type_vector, (4, 1, 2, mvx.MPI_SHORT), vec(4, 1, 2, 2)),
    ]
    stream = torch.cuda.current_stream()
    for name, ctor, args, blocks in cases:
        rc, h = ctor(*args)
        assert rc == 0 and mvx.MPI_Type_commit(h) == 0, name
        ext = mvx.MPI_Type_extent(h)[1]
        size = mvx.MPI_Type_size(h)[1]
        n = SPAN // ext
        sets = []
        for _ in range(2):
            origin = torch.randint(0, 1 << 30, ((n * ext + 3) // 4 + 64,), dtype=torch.int32, device="cuda")
            packed = torch.empty(((n * size + 3) // 4 + 64,), dtype=torch.int32, device="cuda")
            sets.append((origin, packed))
        touched = lines_touched(blocks, ext, n)
        for direction in ("pack", "unpack"):
            def launch(i):
                o, p = sets[i % 2]
                if direction == "pack":
                    rc = mvx.type_pack(h, o, p, n, stream)
                else:
                    rc = mvx.type_unpack(h, p, o, n, stream)
                assert rc == 0, (name, rc)
            for i in range(2):
                launch(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record(stream)
            for i in range(reps):
                launch(i)
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            alg = 2 * n * size
            out = {"type": name, "dir": direction, "elements": n, "extent": ext, "size": size,
                   "packed_bytes": n * size, "us": round(us, 2),
                   "alg_GBs": round(alg / (us * 1e-6) / 1e9, 1), "alg_frac": round(alg / (us * 1e-6) / 1e9 / PEAK, 4)}
            if touched is not None:
                lb = touched + n * size          # lines of the span read (pack) or written (unpack)
                out["line_GBs"] = round(lb / (us * 1e-6) / 1e9, 1)
                out["line_frac"] = round(lb / (us * 1e-6) / 1e9 / PEAK, 4)
                if direction == "unpack":
                    # what DRAM moves when the hole bytes of partly written
                    # lines must be kept: every touched line read and written
                    # (by the memory on a byte-masked store, by the kernel in
                    # MVX_UNPACK_MERGE's whole-word unpack)
                    rmw = 2 * touched + n * size
                    out["rmw_GBs"] = round(rmw / (us * 1e-6) / 1e9, 1)
                    out["rmw_frac"] = round(rmw / (us * 1e-6) / 1e9 / PEAK, 4)
            out["merge"] = os.environ.get("MVX_UNPACK_MERGE", "1") != "0"
            print(json.dumps(out), flush=True)
        del sets
        torch.cuda.empty_cache()
        mvx.MPI_Type_free(h)


if __name__ == "__main__":
    main()
