#!/usr/bin/env python3
"""Tuning probe for the k-leaf combine kernel (config-3 shape: tree k = 8,
SUM f32, 8 x 32 MiB): does the placement of the leaves in HBM (separate
allocations / back-to-back slots as the staging pool lays them out / slots
staggered by a few KiB) or the grid size change the kernel rate?

Prints one JSON line per variant (HIP events on the launch stream, 4 buffer
sets rotated so no step is served from the Infinity Cache).
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MIB = 1 << 20


def main():
    import torch
    mvx = importlib.import_module("mvapich-cce_amd")
    k, leaf = 8, 32 * MIB
    n = leaf // 4
    stream = torch.cuda.current_stream()

    def layout(kind, sets=4):
        out = []
        for _ in range(sets):
            if kind == "separate":
                leaves = [torch.rand(n, device="cuda") for _ in range(k)]
            else:
                stagger = kind if isinstance(kind, int) else \
                    {"slots": 0, "stagger4k": 4096, "stagger64k": 65536 + 256, "stagger1m": MIB + 4096}[kind]
                big = torch.rand((k * (leaf + stagger * k)) // 4 + 1024, device="cuda")
                base = big.data_ptr()
                ptrs = [base + q * (leaf + stagger) for q in range(k)]
                leaves = (big, ptrs)
            dst = torch.empty(n, device="cuda")
            out.append((leaves, dst))
        return out

    def time_it(bufs, reps=30):
        def launch(i):
            leaves, dst = bufs[i % len(bufs)]
            srcs = leaves[1] if isinstance(leaves, tuple) else leaves
            assert mvx.op_combine(102, 10, srcs, dst, n, shape=0, stream=stream) == 0
        for i in range(4):
            launch(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(reps):
            launch(i)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    alg = (k + 1) * leaf
    sweep = "sweep" in sys.argv[1:] or "fine" in sys.argv[1:]
    kinds = [4096, 0, 512, 1536, 2560, 3072, 3584, 4096, 4352, 4608, 5120, 6144, 10240, 12288, 4096] \
        if "fine" in sys.argv[1:] else \
        ["slots", 256, 1024, 2048, 4096, 6144, 8192, 12288, 16384, 32768, "slots", 4096] if sweep else \
        ["separate", "slots", "stagger4k", "stagger64k", "stagger1m"]
    for kind in kinds:
        bufs = layout(kind)
        for cap in ((0,) if sweep else (0, 2048, 1024)):
            mvx.set_launch(cap if cap else (1 << 20), 0)
            us = time_it(bufs)
            print(json.dumps({"layout": kind, "block_cap": cap or "one-pass", "kernel_us": round(us, 2),
                              "GBps": round(alg / us / 1e3, 1), "hbm_frac": round(alg / us / 1e3 / 8000, 4)}),
                  flush=True)
        mvx.set_launch(1 << 20, 0)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
