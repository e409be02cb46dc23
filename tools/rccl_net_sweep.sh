#!/bin/bash
# Seeded random sweeps (tests/mp_worker.py "random": collective, op x type
# with the undefined pairs, count, root, exchange variant, device or host
# buffers) on RCCL communicators of WORLDS ranks sharing the box's one GPU,
# RCCL's socket transport moving the bytes (transport.rccl_net_env); every
# rank's code and recvbuf against the oracle.  One JSON line per world.
#   MVX_MP_CASES=300 WORLDS="3 5 6 8" tools/rccl_net_sweep.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MVX_MP_CASES=${MVX_MP_CASES:-300}
export WORLDS=${WORLDS:-3 5 6 8}
timeout -k 10 1000 python -u - <<'PY'
import json, os, sys
sys.path.insert(0, "tests")
import test_gpu_multiproc as T
for w in map(int, os.environ["WORLDS"].split()):
    reps = T._launch(w, "rccl-net", "random", 900)
    fails = [f for r in reps for f in r["fails"]]
    print(json.dumps({"world": w, "transport": "rccl-net", "cases": reps[0]["checked"],
                      "ranks_checked": len(reps), "fails": len(fails), "first_fails": fails[:3]}), flush=True)
    if fails:
        sys.exit(1)
PY
