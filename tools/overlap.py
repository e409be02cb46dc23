"""Does the PIPE exchange overlap its combines with RCCL's transfers?  Reads
one rank's rocprofv3 kernel trace (CSV) and reports, for every combine
kernel (mvx::k_*), the time during which an RCCL kernel of the same process
ran concurrently on another queue, plus the P2P reference: the same numbers
for a run whose combines are stream-ordered between the transfers (none
expected).  Used by tools/prof_pipe_overlap.sh.
  python3 tools/overlap.py TRACE.csv [label]  ->  one JSON line
"""
import csv
import json
import sys


def main(path, label=""):
    rows = list(csv.DictReader(open(path)))
    comb, rccl = [], []
    for r in rows:
        name = r["Kernel_Name"]
        span = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Stream_Id"])
        if "mvx::k_" in name:
            comb.append(span)
        elif "nccl" in name.lower():
            rccl.append(span)
    rccl.sort()
    over, overlapped, total = 0, 0, 0
    for s, e, q, st in comb:
        total += e - s
        o = 0
        for rs, re_, rq, rst in rccl:
            if rs >= e:
                break
            if re_ > s and (rq, rst) != (q, st):
                o += min(e, re_) - max(s, rs)
        o = min(o, e - s)
        over += o
        overlapped += o > 0
    print(json.dumps({"label": label, "combines": len(comb), "rccl_kernels": len(rccl),
                      "combines_overlapped": overlapped, "combine_us": round(total / 1e3, 1),
                      "combine_us_under_rccl": round(over / 1e3, 1),
                      "fraction_hidden": round(over / total, 3) if total else None,
                      "combine_queues": sorted({c[2] for c in comb}), "rccl_queues": sorted({c[2] for c in rccl})}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
