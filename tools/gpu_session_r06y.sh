# Round-6 session y: seeded sweeps on the final build -- the op functions
# with the registration cache on and operands sharing pages (new), the
# derived-type collective sweep (40 batches), 3000 collective cases and
# 1000 op-function cases with fresh seeds.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
MVX_FUZZ_REG_BATCHES=8 MVX_FUZZ_SEED=9090909 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "random_op_functions_registered" > gpurun_out/r06y_fuzz_registered.log 2>&1 || { tail -40 gpurun_out/r06y_fuzz_registered.log; exit 1; }
tail -n 1 gpurun_out/r06y_fuzz_registered.log
MVX_FUZZ_DT_BATCHES=40 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_types.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "random_derived_sweep" > gpurun_out/r06y_derived_sweep_40.log 2>&1 || { tail -30 gpurun_out/r06y_derived_sweep_40.log; exit 1; }
tail -n 1 gpurun_out/r06y_derived_sweep_40.log
SEED=8080808 bash tools/fuzz_sweep_big_r05.sh || exit 1
cp gpurun_out/fuzz_sweep_big.log gpurun_out/r06y_fuzz_sweep_3000_seed8080808.log
SEED=8181818 bash tools/fuzz_ops_big_r05.sh || exit 1
cp gpurun_out/fuzz_ops_big.log gpurun_out/r06y_fuzz_ops_1000_seed8181818.log
