# Programs over 3-4 leaves on KMAX = 4 kernels at U = 2 (MVX_PROG4, default
# on): the op / body parity suites, then tools/bench_kernels.py ks with and
# without, interleaved twice.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_body.py tests/test_gpu_ops.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/prog4_tests.log 2>&1 || { tail -40 gpurun_out/prog4_tests.log; exit 1; }
tail -1 gpurun_out/prog4_tests.log
: > gpurun_out/prog4_ab.jsonl
for pass in 1 2; do for on in 0 1; do
  MVX_PROG4=$on timeout -k 10 200 python3 tools/bench_kernels.py ks 2>/dev/null | grep '"K-' | sed "s/^{/{\"prog4\": $on, /" >> gpurun_out/prog4_ab.jsonl || exit 1
done; done
