#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes for one kernel into a committed JSON.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: rocprofv3
reports both in KiB, and on gfx950 FETCH_SIZE counts exactly half the bytes
of a wide coalesced streaming read (MI355X_MICROARCH.md, section HBM), so the
read side is doubled before it is compared with a byte count.

usage: pmc_summary.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR KERNEL_TAG VECTOR_BYTES ALG_BYTES OUT.json
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter, substr):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter or substr not in row.get("Kernel_Name", ""):
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, substr, tag, vbytes, abytes, out = sys.argv[1:8]
    fetch = per_dispatch(fdir, "FETCH_SIZE", substr)
    write = per_dispatch(wdir, "WRITE_SIZE", substr)
    if not fetch or not write:
        sys.exit("no dispatches of %r found" % substr)
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    hbm = (2 * f_kib + w_kib) * 1024
    doc = {"kernel_tag": tag, "kernel_match": substr, "vector_bytes": int(vbytes),
           "dispatches": {"fetch": len(fetch), "write": len(write)},
           "FETCH_SIZE_kib_median": f_kib, "WRITE_SIZE_kib_median": w_kib,
           "hbm_bytes_per_launch": int(hbm), "alg_bytes_per_launch": int(abytes),
           "traffic_over_algorithmic": round(hbm / int(abytes), 4),
           "correction": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = half the streamed bytes)"}
    with open(out, "w") as fo:
        json.dump(doc, fo, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
