#!/bin/bash
# Rehearse the N>1 bench legs at their FULL BASELINE sizes on ONE GPU
# (c3 256 MiB x 8 ranks, c4 1 GiB x 4, c5 512 MiB x 8): the reference run,
# digests and every exchange variant at the sizes the driver's 8-GPU node
# will use.  TRANSPORT=host (default: gloo moves the blocks) or rccl-net
# (RCCL communicators, its socket transport moves them).  Slow; few steps.
#   [TRANSPORT=rccl-net] tools/rehearse_full.sh [cfg ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cfgs=${*:-c3 c4 c5}
tr=${TRANSPORT:-host}
for cfg in $cfgs; do
  np=8; [ $cfg = c4 ] && np=4
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus $np --transport $tr --config $cfg --steps 2 --warmup 1 --tune-steps 1 > gpurun_out/full_${tr}_$cfg.log 2>&1 || { tail -30 gpurun_out/full_${tr}_$cfg.log; exit 1; }
  grep '"metric"' gpurun_out/full_${tr}_$cfg.log > gpurun_out/full_${tr}_$cfg.jsonl
  python3 -c "import sys,json; d=json.load(open('gpurun_out/full_${tr}_$cfg.jsonl')); print('$cfg', d['n_gpus'], d['config']['vector_bytes_per_rank'], d['parity'], d['config']['exchange'], {k:(v['ran'],v['parity']) for k,v in d['config']['exchange_tuning'].items()}, d['cpu_baseline'], [(o['config'], o['parity']) for o in d.get('other_configs', [])])"
done
