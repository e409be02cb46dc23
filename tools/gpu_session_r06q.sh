# Round-6 session q: seeded sweeps on the final tile kernels -- 40 batches
# of the derived-type collective sweep (whole recv buffers compared), and a
# 3000-case collective sweep with a fresh seed.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
MVX_FUZZ_DT_BATCHES=40 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_types.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "random_derived_sweep" > gpurun_out/r06q_derived_sweep_40.log 2>&1 || { tail -30 gpurun_out/r06q_derived_sweep_40.log; exit 1; }
tail -1 gpurun_out/r06q_derived_sweep_40.log
SEED=7070707 bash tools/fuzz_sweep_big_r05.sh || exit 1
cp gpurun_out/fuzz_sweep_big.log gpurun_out/r06q_fuzz_sweep_3000_seed7070707.log
