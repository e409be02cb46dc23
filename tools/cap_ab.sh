#!/bin/bash
# A/B of the residency cap (MVX_CAP_*: resident blocks per CU for the
# non-temporal launches) on the BASELINE combine shapes, interleaved on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in default uncapped progcap; do
    case $v in
      default) envs="" ;;
      uncapped) envs="MVX_CAP_APPLY=0 MVX_CAP_TREE=0 MVX_CAP_PROG=0" ;;
      progcap) envs="MVX_CAP_PROG=3" ;;
    esac
    env $envs timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/cap_${v}_$r.jsonl 2>> gpurun_out/cap_ab.err || exit 1
    echo "-- $v $r"; python3 -c "
import json,sys
for l in open('gpurun_out/cap_${v}_$r.jsonl'):
    d=json.loads(l); print(d['config'], d['kernel_us'], d['hbm_frac'])
"
  done
done
