# Round-6 session yy: the seeded sweeps of session y again with fresh seeds
# on the final build (chain body with a run-time leaf count, chunk tables,
# LDS swizzle).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
MVX_FUZZ_REG_BATCHES=8 MVX_FUZZ_SEED=9191919 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "random_op_functions_registered" > gpurun_out/r06yy_fuzz_registered.log 2>&1 || { tail -40 gpurun_out/r06yy_fuzz_registered.log; exit 1; }
tail -n 1 gpurun_out/r06yy_fuzz_registered.log
MVX_FUZZ_DT_BATCHES=40 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_types.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "random_derived_sweep" > gpurun_out/r06yy_derived_sweep_40.log 2>&1 || { tail -30 gpurun_out/r06yy_derived_sweep_40.log; exit 1; }
tail -n 1 gpurun_out/r06yy_derived_sweep_40.log
SEED=8282828 bash tools/fuzz_sweep_big_r05.sh || exit 1
cp gpurun_out/fuzz_sweep_big.log gpurun_out/r06yy_fuzz_sweep_3000_seed8282828.log
SEED=8383838 bash tools/fuzz_ops_big_r05.sh || exit 1
cp gpurun_out/fuzz_ops_big.log gpurun_out/r06yy_fuzz_ops_1000_seed8383838.log
