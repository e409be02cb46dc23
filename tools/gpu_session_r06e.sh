# Round-6 session e: the N = 8 leg at full size on one GPU over RCCL's socket
# transport (rccl-net), self-launched (bench.py starts its 8 workers) with
# the graph variants too, then in the driver's torchrun form.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --gpus 8 --transport rccl-net --config c3 --steps 2 --warmup 1 --tune-steps 1 --graphs \
  > gpurun_out/r06e_n8_self.json 2> gpurun_out/r06e_n8_self.err || { tail -30 gpurun_out/r06e_n8_self.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06e_n8_self.json')); print(d['n_gpus'], d['parity'], d['config']['exchange'], {k:(v['ran'],v['parity'],v['ms_per_step']) for k,v in d['config']['exchange_tuning'].items()})"
TRANSPORT=rccl-net timeout -k 10 560 bash tools/rehearse_full.sh c3 || exit 1
