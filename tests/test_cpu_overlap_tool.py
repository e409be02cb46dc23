"""CPU: tools/overlap.py -- the combine time it counts as under an RCCL
kernel, on a synthetic kernel trace (the rocprofv3 CSV columns it reads)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kind", "Queue_Id", "Stream_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for q, st, name, s, e in rows:
            w.writerow(["KERNEL_DISPATCH", q, st, name, s, e])


def _run(path):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "overlap.py"), str(path), "x"],
                         capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def test_overlap_counts_only_other_queue_time(tmp_path):
    p = tmp_path / "t.csv"
    _trace(p, [
        (4, 7, "void rcclGenericKernel<2, false>(ncclDevComm*)", 0, 1000),
        (5, 8, "void mvx::k_combine<2, float, 2, 4, 1, 0>(mvx::Params)", 900, 1100),     # 100 of 200 under
        (4, 7, "void rcclGenericKernel<2, false>(ncclDevComm*)", 1100, 2000),
        (5, 8, "void mvx::k_tree_body<2, float, 8, 2>(mvx::BodyParams)", 1200, 1300),   # all 100 under
        (4, 7, "void mvx::k_combine<2, float, 2, 4, 1, 0>(mvx::Params)", 2000, 2100),   # after: none
    ])
    d = _run(p)
    assert d["combines"] == 3 and d["rccl_kernels"] == 2
    assert d["combine_us"] == 0.4 and d["combine_us_under_rccl"] == 0.2
    assert d["combines_overlapped"] == 2 and d["fraction_hidden"] == 0.5
    assert d["combine_queues"] == ["4", "5"] and d["rccl_queues"] == ["4"]


def test_same_stream_is_never_overlap(tmp_path):
    """a combine on the transfers' own stream cannot run beside them"""
    p = tmp_path / "t.csv"
    _trace(p, [(4, 7, "ncclKernel", 0, 1000), (4, 7, "mvx::k_combine<2, float, 2, 4, 1, 0>", 500, 600)])
    assert _run(p)["combine_us_under_rccl"] == 0.0
