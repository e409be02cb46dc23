#!/bin/bash
# A/B of the grid size of the combine kernels (MVX_BLOCK_CAP: at most this
# many blocks, grid-stride beyond; 0 = one block per work unit, the default)
# on the BASELINE combine shapes, interleaved on one box.  512 = one wave of
# resident blocks at the trees' 2-per-CU cap (256 CUs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for cap in 0 512 1024 2048; do
    if [[ $cap == 0 ]]; then envs=""; else envs="MVX_BLOCK_CAP=$cap"; fi
    env $envs timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/grid_${cap}_$r.jsonl 2>> gpurun_out/grid_ab.err || exit 1
    echo "-- cap $cap run $r"; python3 -c "
import json,sys
for l in open('gpurun_out/grid_${cap}_$r.jsonl'):
    d=json.loads(l); print(d['config'], d['kernel_us'], d['hbm_frac'])
"
  done
done
