"""Does a host-buffer rank overlap its PCIe copies with the collective?
Reads one rank's rocprofv3 output directory (--kernel-trace
--memory-copy-trace, CSV) and reports the busy time of each stream of work
-- host-to-device copies, device-to-host copies (SDMA, or HIP's blit
kernels, which it used for the slices' D2H), the collective's kernels (RCCL
transfers and the combines) -- the time covered by any of them, and how much of each ran
while another kind was running.  overlap_factor = (sum of the three busy
times) / (time covered by any): 1.0 when they run one after another, up to
3.0 when all three always run together.  Used by tools/prof_host_multi.sh.

  python3 tools/host_overlap.py RANK_DIR [label]  ->  one JSON line
"""
import csv
import glob
import json
import os
import sys


def _rows(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main(d, label=""):
    copies = _rows(d, "*memory_copy_trace.csv")
    kernels = _rows(d, "*kernel_trace.csv")
    h2d, d2h, ker = [], [], []
    for r in copies:
        way = (r.get("Direction") or r.get("Operation") or r.get("Kind") or "").upper()
        span = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        if "HOST_TO_DEVICE" in way:
            h2d.append(span)
        elif "DEVICE_TO_HOST" in way:
            d2h.append(span)
    blit = []
    for r in kernels:
        span = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        name = r["Kernel_Name"]
        if "copyBuffer" in name:          # HIP's blit-kernel copies (it ran the slices' D2H this way)
            blit.append(span)
        elif "mvx::" in name or "ncclDevKernel" in name or "rccl" in name.lower():
            ker.append(span)             # the collective: RCCL transfers and the combines
    H, D, K = union(h2d), union(d2h + blit), union(ker)
    anyb = union(H + D + K)
    tot = length(anyb)
    res = {"label": label, "h2d_copies": len(h2d), "d2h_copies": len(d2h), "blit_copies": len(blit),
           "collective_kernels": len(ker),
           "h2d_ms": round(length(H) / 1e6, 3), "d2h_ms": round(length(D) / 1e6, 3),
           "kernel_ms": round(length(K) / 1e6, 3), "any_ms": round(tot / 1e6, 3),
           "overlap_factor": round((length(H) + length(D) + length(K)) / tot, 3) if tot else None,
           "h2d_under_d2h_frac": round(length(intersect(H, D)) / length(H), 3) if H else None,
           "kernel_under_copies_frac": round(length(intersect(K, union(H + D))) / length(K), 3) if K else None}
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
