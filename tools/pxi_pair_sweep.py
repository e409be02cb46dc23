#!/usr/bin/env python3
"""Seeded random sweep of the MPI_LONG_DOUBLE_INT MAXLOC / MINLOC lane-pair
body kernel (k_pxi_loc_body) against the oracle's x87: tree over k = 4 or 8
leaves, sizes that take the non-temporal body path, a fraction of elements
with equal values across leaves (the loc = min rule).  One JSON line per
case, then a summary.   python tools/pxi_pair_sweep.py [CASES]"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import numpy as np
    import test_gpu_body as B
    from plan_exec import SHAPE_TREE
    mvx = importlib.import_module("mvapich-cce_amd")
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    bad = 0
    for i in range(cases):
        rng = np.random.default_rng(9000 + i)
        k = int(rng.choice([4, 8]))
        op = int(rng.choice([110, 111]))
        n = int(rng.integers(420_000, 800_000))
        ties = float(rng.choice([0.0, 0.3, 0.9]))
        sym, got, ref = B._run(mvx, op, 22, k, SHAPE_TREE, n, seed=1000 + i, ties=ties)
        ok = bool(np.array_equal(got, ref)) and sym.startswith("k_pxi_loc_body<")
        bad += not ok
        print(json.dumps({"case": i, "op": op, "k": k, "n": n, "ties": ties, "kernel": sym, "bit_exact": ok}),
              flush=True)
    print(json.dumps({"cases": cases, "mismatches": bad}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
