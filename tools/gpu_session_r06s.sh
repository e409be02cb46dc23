# Round-6 session s: buffers under a neighbour's registration -- the probe,
# the registration-cache tests, the host-buffer table (its op_registered
# rows found the case), the multi-process host suites and the derived types.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/shadow_probe > gpurun_out/r06s_shadow_probe.json || exit 1
cat gpurun_out/r06s_shadow_probe.json
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 500 $PT -s tests/test_gpu_host_register.py > gpurun_out/r06s_reg.log 2>&1 || { tail -60 gpurun_out/r06s_reg.log; exit 1; }
grep -E "PASSED|FAILED|mode" gpurun_out/r06s_reg.log | cut -c1-200
bash tools/gpu_round.sh host > gpurun_out/r06s_host.log 2>&1 || { tail -30 gpurun_out/r06s_host.log; exit 1; }
grep -c '"case"' gpurun_out/bench_host.jsonl
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_types.py tests/test_gpu_derived.py tests/test_gpu_exec.py tests/test_gpu_userops.py > gpurun_out/r06s_suites.log 2>&1 || { tail -40 gpurun_out/r06s_suites.log; exit 1; }
tail -1 gpurun_out/r06s_suites.log
