"""tools/scale_vs_model.py: bench's N > 1 lines read against the per-phase
model registered in DESIGN.md section 6 (for the driver's SCALE record)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(n, ms, a, b, c):
    return {"metric": "m", "n_gpus": n, "ms_per_step": ms,
            "config": {"workload": "c3: MPI_Allreduce ...", "exchange_ran": "p2p"},
            "roofline": {"frac": 0.8, "phases": {"A_ms": a, "B_ms": b, "C_ms": c,
                                                 "A_GBs_per_rank": {"per_link": 150.0, "link_frac": 0.98}}}}


def test_scale_lines_against_model(tmp_path):
    rec = {"runs": [json.dumps(_line(8, 0.55, 0.25, 0.05, 0.24)), {"bench": _line(2, 2.0, 0.9, 0.07, 0.9)},
                    {"metric": "m", "n_gpus": 1, "ms_per_step": 0.125, "config": {"workload": "config2"}}]}
    f = tmp_path / "scale.json"
    f.write_text(json.dumps(rec))
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "scale_vs_model.py"), str(f)],
                                  text=True)
    rows = [r for r in out.splitlines() if r.startswith("| 2") or r.startswith("| 8")]
    assert len(rows) == 2, out                          # N = 1 left out
    assert rows[0].startswith("| 2 | c3 | p2p | 2.0 | 1.82 | 1.10 |"), rows[0]
    assert "0.25 / 0.219 (1.14)" in rows[1] and "150.0 (0.98)" in rows[1], rows[1]


def test_scale_json_lines_file(tmp_path):
    f = tmp_path / "lines.jsonl"
    f.write_text(json.dumps(_line(4, 1.0, 0.44, 0.05, 0.44)) + "\nnoise\n")
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "scale_vs_model.py"), str(f)],
                                  text=True)
    assert "| 4 | c3 | p2p | 1.0 | 0.93 | 1.08 |" in out
