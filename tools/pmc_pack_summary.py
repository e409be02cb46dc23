#!/usr/bin/env python3
"""Median HBM bytes per dispatch of the pack / unpack kernels from two
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over tools/bench_pack.py.

bench_pack.py launches, per case in its order, 12 pack then 12 unpack
dispatches; the pack-engine kernels (k_pack_units, k_pack, k_pack_tiles, k_unpack_merge)
are taken in dispatch order and cut into groups of 12.  FETCH_SIZE is
doubled (gfx950 tallies 128-byte requests at 64 B, MI355X_MICROARCH.md; exact
for 16-B/lane streams); the counters are KiB, printed as MB (1e6 B).

  python3 tools/pmc_pack_summary.py FETCH_DIR WRITE_DIR BENCH_JSONL > out.txt
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("k_pack_units", "k_pack<", "k_unpack_merge", "k_pack_tiles")


def rows(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] == counter and any(k in r["Kernel_Name"] for k in KERNELS):
                out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    out.sort()
    return out


def main():
    fetch, write = rows(sys.argv[1], "FETCH_SIZE"), rows(sys.argv[2], "WRITE_SIZE")
    cases = [json.loads(line) for line in open(sys.argv[3])]
    assert len(fetch) == len(write) == 12 * len(cases), (len(fetch), len(write), len(cases))
    print("# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/bench_pack.py on MI355X, "
          "median of 12 dispatches per (type, direction); FETCH_SIZE x2, counters in KiB, MB = 1e6 B")
    for g, c in enumerate(cases):
        f = fetch[12 * g:12 * g + 12]
        w = write[12 * g:12 * g + 12]
        name = f[0][1][:48]
        fm = 2 * statistics.median(x[2] for x in f) * 1024 / 1e6
        wm = statistics.median(x[2] for x in w) * 1024 / 1e6
        print("%-48s %-6s %-48s fetch_x2 %8.1f MB  write %8.1f MB  us %7.2f" % (c["type"], c["dir"], name, fm, wm,
                                                                             c["us"]))


if __name__ == "__main__":
    main()
