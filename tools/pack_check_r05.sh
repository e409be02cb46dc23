# The unit pack / unpack kernels (csrc/mvx_dtype.hip k_pack_units): the
# datatype parity suites, then tools/bench_pack.py with the unit kernels
# (default) and with the piece kernel only (MVX_PACK_UNITS=0).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_types.py tests/test_gpu_derived.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 || { tail -40 gpurun_out/pack_tests.log; exit 1; }
tail -2 gpurun_out/pack_tests.log
timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/bench_pack_units.jsonl 2> gpurun_out/bp.err || { tail -5 gpurun_out/bp.err; exit 1; }
MVX_PACK_UNITS=0 timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/bench_pack_pieces.jsonl 2> gpurun_out/bp.err || { tail -5 gpurun_out/bp.err; exit 1; }
