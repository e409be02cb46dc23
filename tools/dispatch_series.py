#!/usr/bin/env python3
"""Per-dispatch durations of one kernel across a bench.py N = 1 run, from a
rocprofv3 --kernel-trace CSV: which launches were the prewarm, the W warmup
steps, the K timed steps, the K evented steps and the parity step, and what
each segment averaged.

  tools/dispatch_series.py TRACE_DIR KERNEL_SUBSTRING K [OUT.json]

bench.py's order at N = 1 is: prewarm (any count), W warmup, K timed, K
evented, 1 parity step -- so the segments are read from the END of the
series, and the count of the prewarm/warmup part is whatever precedes them.
"""
import csv
import glob
import json
import os
import statistics
import sys


def load(trace_dir, sub):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit("no kernel_trace.csv under %s" % trace_dir)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if sub in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def seg(rows):
    d = [(e - s) / 1e3 for s, e, _ in rows]
    if not d:
        return None
    return {"n": len(d), "mean_us": round(statistics.mean(d), 2), "median_us": round(statistics.median(d), 2),
            "min_us": round(min(d), 2), "max_us": round(max(d), 2), "us": [round(x, 2) for x in d]}


def main():
    trace_dir, sub, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = load(trace_dir, sub)
    if len(rows) < 2 * k + 1:
        sys.exit("only %d dispatches of %r" % (len(rows), sub))
    parity = rows[-1:]
    evented = rows[-(k + 1):-1]
    timed = rows[-(2 * k + 1):-(k + 1)]
    before = rows[:-(2 * k + 1)]
    # gaps between consecutive timed dispatches (GPU idle inside the timed region)
    gaps = [(timed[i + 1][0] - timed[i][1]) / 1e3 for i in range(len(timed) - 1)]
    span_us = (timed[-1][1] - timed[0][0]) / 1e3
    out = {"kernel": rows[0][2], "dispatches": len(rows),
           "prewarm_and_warmup": seg(before), "timed": seg(timed), "evented": seg(evented),
           "parity": seg(parity),
           "timed_span_us": round(span_us, 2), "timed_span_per_step_us": round(span_us / k, 2),
           "timed_gap_us": {"mean": round(statistics.mean(gaps), 2), "max": round(max(gaps), 2)} if gaps else None}
    if out["prewarm_and_warmup"]:
        b = out["prewarm_and_warmup"]["us"]
        out["prewarm_and_warmup"]["first_10_us"] = b[:10]
        out["prewarm_and_warmup"]["last_10_us"] = b[-10:]
        del out["prewarm_and_warmup"]["us"]
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
