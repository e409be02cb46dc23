# The x87 add's general path out of line (mvx_xf80.h add_general): the x87
# parity tests, then the x87 kernel rates (tools/bench_kernels.py x87).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_body.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "x87 or long_double or every_pair or 12 or LDI or 22" > gpurun_out/x87_tests.log 2>&1 \
  || { tail -40 gpurun_out/x87_tests.log; exit 1; }
tail -1 gpurun_out/x87_tests.log
timeout -k 10 300 python3 tools/bench_kernels.py x87 > gpurun_out/bench_kernels_x87_cold.jsonl 2>/dev/null || exit 1
cat gpurun_out/bench_kernels_x87_cold.jsonl
