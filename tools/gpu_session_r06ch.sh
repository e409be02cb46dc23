# Round-6 session ch: chains of 5-7 leaves on the 8-leaf chain body with a
# run-time leaf count: the body and collective suites, then the leaf-count
# sweep (tools/bench_kernels.py ks) with MVX_CHAIN_RT=1 / 0, two passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_body.py tests/test_gpu_coll.py > gpurun_out/r06ch_pytest.log 2>&1 || { tail -40 gpurun_out/r06ch_pytest.log; exit 1; }
tail -n 1 gpurun_out/r06ch_pytest.log
: > gpurun_out/r06ch_ks.jsonl
for pass in 1 2; do for rt in 1 0; do
  MVX_CHAIN_RT=$rt timeout -k 10 300 python3 tools/bench_kernels.py ks > gpurun_out/r06ch_ks.tmp 2> gpurun_out/r06ch_ks.err || { tail -20 gpurun_out/r06ch_ks.err; exit 1; }
  grep '^{' gpurun_out/r06ch_ks.tmp | sed "s/^{/{\"chain_rt\": $rt, \"pass\": $pass, /" >> gpurun_out/r06ch_ks.jsonl
done; done
python3 -c "
import json
for l in open('gpurun_out/r06ch_ks.jsonl'):
    d = json.loads(l)
    if 'chain' in d['config']: print(d['chain_rt'], d['pass'], d['config'], d['kernel_us'], d['hbm_frac'])"
