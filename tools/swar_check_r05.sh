# The SWAR 1-byte chunk op and the MPI_LONG_DOUBLE_INT lane-pair apply body:
# the op / body parity tests, then every op x type apply kernel's rate.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_body.py tests/test_gpu_ops.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/swar_tests.log 2>&1 || { tail -40 gpurun_out/swar_tests.log; exit 1; }
tail -2 gpurun_out/swar_tests.log
timeout -k 10 400 python3 tools/bench_kernels.py all > gpurun_out/bench_kernels_all_swar.jsonl 2> gpurun_out/bench_kernels_all_swar.err \
  || { tail -5 gpurun_out/bench_kernels_all_swar.err; exit 1; }
wc -l gpurun_out/bench_kernels_all_swar.jsonl
