# Zero copy in the op functions (csrc/mvx_hostop.c): the parity tests of the
# host-operand paths, then an interleaved A/B of MVX_HOST_ZEROCOPY=0 (the DMA
# pipeline through HBM) against 1 (the kernel reads / writes page-locked
# operands and the pinned bounce slots of pageable ones in place), two
# passes each, tools/bench_host.py.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "pinned_zero_copy or host_buffers" > gpurun_out/zc_tests.log 2>&1 || { tail -30 gpurun_out/zc_tests.log; exit 1; }
tail -2 gpurun_out/zc_tests.log
out=gpurun_out/zc_ab.jsonl; : > $out
for pass in 1 2; do for zc in 0 1; do
  MVX_HOST_ZEROCOPY=$zc timeout -k 10 120 python3 tools/bench_host.py --min-mib ${MIN_MIB:-0} --cases ${CASES:-op_pinned,op_registered} \
    > gpurun_out/zc.tmp 2>&1 || { cat gpurun_out/zc.tmp; exit 1; }
  grep '^{' gpurun_out/zc.tmp | sed "s/^{/{\"zerocopy\": $zc, \"pass\": $pass, /" >> $out
done; done
cat $out
