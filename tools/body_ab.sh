#!/bin/bash
# A/B of the body kernels' loop form (MVX_BODY_FULL=0: bounds-tested chunks
# always; default 1: whole-iteration launches skip the tests) crossed with the
# grid size (MVX_BLOCK_CAP: 0 = a block per work unit, 512 = one wave of
# resident blocks at the trees' 2-per-CU cap) on the BASELINE combine shapes,
# interleaved on one box (tools/bench_kernels.py, HIP events, rotating sets).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for full in 0 1; do
    for cap in 0 512; do
      envs="MVX_BODY_FULL=$full"
      [[ $cap != 0 ]] && envs="$envs MVX_BLOCK_CAP=$cap"
      env $envs timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/body_f${full}_c${cap}_$r.jsonl 2>> gpurun_out/body_ab.err || exit 1
      python3 -c "
import json
rows = [json.loads(l) for l in open('gpurun_out/body_f${full}_c${cap}_$r.jsonl')]
print('full=$full cap=$cap run=$r', ' '.join('%s %.2f us %.4f' % (d['config'], d['kernel_us'], d['hbm_frac']) for d in rows))
"
    done
  done
done
