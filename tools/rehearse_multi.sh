#!/bin/bash
# Rehearse the N>1 bench legs (c3 at 8 ranks, c4 at 4, c5 at 8) on ONE GPU
# through the host transport: small vectors, every exchange variant, parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in c3 c4 c5; do
  np=8; [ $cfg = c4 ] && np=4
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $np --transport host --config $cfg --steps 3 --warmup 1 --mib 16 --tune-steps 1 > gpurun_out/mp8_$cfg.log 2>&1 || { tail -30 gpurun_out/mp8_$cfg.log; exit 1; }
  grep '"metric"' gpurun_out/mp8_$cfg.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$cfg', d['n_gpus'], d['value'], d['parity'], d['config']['exchange'], {k:v['parity'] for k,v in d['config']['exchange_tuning'].items()}, d['cpu_baseline']['cores'], d['roofline']['phases'])"
done
cat gpurun_out/mp8_c3.log gpurun_out/mp8_c4.log gpurun_out/mp8_c5.log | grep '"metric"' > gpurun_out/rehearse_multi_host.jsonl
