#!/usr/bin/env python3
"""Read bench.py's N > 1 lines (the driver's SCALE run, or any JSON lines /
JSON files holding them) against the per-phase model registered in
DESIGN.md section 6 before any multi-GPU run: a fully connected node, one
153 GB/s xGMI link per pair, phases A / C one block per link, phase B at the
combine's measured HBM rate.

  python3 tools/scale_vs_model.py SCALE_rNN.json [more.json ...]

One markdown row per line: N, config, the variant that ran, the step time
against the model's p2p total, and phase by phase (A, B, C) measured against
modelled milliseconds, with A / C's per-link rate.  A phase well over its
model with a low link_frac points at RCCL's transfers; phases near the model
with a total far over it point at the gaps between phases.
"""
import json
import sys

# DESIGN.md section 6, "Expected time per phase" (ms): (A, B, C, p2p total)
MODEL = {
    ("c3", 2): (0.877, 0.064, 0.877, 1.82), ("c3", 4): (0.439, 0.053, 0.439, 0.93),
    ("c3", 8): (0.219, 0.049, 0.219, 0.49),
    ("c4", 2): (3.51, 0.25, None, 3.76), ("c4", 4): (1.75, 0.20, None, 1.96), ("c4", 8): (0.877, 0.19, None, 1.07),
    ("c5", 2): (1.75, 0.13, 1.75, 3.64), ("c5", 4): (0.877, 0.11, 0.877, 1.87), ("c5", 8): (0.439, 0.095, 0.439, 0.97),
}


def lines_from(path):
    """bench lines from a file of JSON lines, a JSON list, or a JSON object
    whose values hold lines (the driver's record)"""
    with open(path) as f:
        text = f.read()
    out = []

    def walk(x):
        if isinstance(x, dict):
            if "metric" in x and "n_gpus" in x:
                out.append(x)
            else:
                for v in x.values():
                    walk(v)
        elif isinstance(x, list):
            for v in x:
                walk(v)
        elif isinstance(x, str) and x.lstrip().startswith("{"):
            try:
                walk(json.loads(x))
            except ValueError:
                pass
    try:
        walk(json.loads(text))
    except ValueError:
        for ln in text.splitlines():
            ln = ln.strip()
            if ln.startswith("{"):
                try:
                    walk(json.loads(ln))
                except ValueError:
                    pass
    return out


def ratio(meas, model):
    return "%.2f" % (meas / model) if meas and model else "-"


def row(d):
    n = d.get("n_gpus")
    cfg = str(d.get("config", {}).get("workload", "")).split(":")[0].strip()
    roof = d.get("roofline") or {}
    ph = roof.get("phases") or {}
    m = MODEL.get((cfg, n))
    ms = d.get("ms_per_step")
    cells = [str(n), cfg, str(d.get("config", {}).get("exchange_ran")), "%s" % ms,
             "%s" % (m[3] if m else "-"), ratio(ms, m[3] if m else None)]
    for i, k in enumerate(("A", "B", "C")):
        meas = ph.get(k + "_ms")
        cells.append("%s / %s (%s)" % (meas, m[i] if m else "-", ratio(meas, m[i] if m else None)))
    for k in ("A", "C"):
        r = ph.get(k + "_GBs_per_rank") or {}
        cells.append("%s (%s)" % (r.get("per_link", "-"), r.get("link_frac", "-")))
    cells.append("%s" % roof.get("frac"))
    return "| " + " | ".join(cells) + " |"


HEADER = ("| N | config | variant | ms/step | model p2p ms | ratio | A ms / model | B ms / model | C ms / model "
          "| A GB/s per link (frac) | C GB/s per link (frac) | busbw frac |\n"
          "|---|---|---|---|---|---|---|---|---|---|---|---|")


def main(paths):
    rows = []
    for p in paths:
        rows += [d for d in lines_from(p) if (d.get("n_gpus") or 1) > 1]
    print(HEADER)
    for d in sorted(rows, key=lambda d: (str(d.get("config", {}).get("workload")), d.get("n_gpus"))):
        print(row(d))
    return 0 if rows else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
