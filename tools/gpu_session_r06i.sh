# Round-6 session i: the driver's N > 1 form (torchrun, default config and
# extra configs) at N = 2 and 4 over rccl-net on the one GPU, this build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29631 \
    bench.py --gpus $n --steps 3 --warmup 1 --tune-steps 2 --transport rccl-net > gpurun_out/r06i_n$n.log 2>&1 || { tail -30 gpurun_out/r06i_n$n.log; exit 1; }
  grep '"metric"' gpurun_out/r06i_n$n.log > gpurun_out/r06i_driver_form_n${n}_rccl_net.json
  python3 -c "import json; d=json.load(open('gpurun_out/r06i_driver_form_n${n}_rccl_net.json')); print($n, d['value'], d['parity'], d['config']['exchange'], [(o['config'], o['parity']) for o in d.get('other_configs', [])])"
done
