# One-off seeded collective sweep after the round-5 kernel changes (SWAR
# 1-byte ops, unit pack kernels, zero copy): 3000 random cases (communicator
# size, collective, op x type including undefined pairs and derived types,
# counts, buffer kinds, exchange variants, user ops) against the oracle.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MVX_FUZZ_CASES=3000 MVX_FUZZ_SEED=${SEED:-777} timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q \
  -p no:cacheprovider --timeout 600 --timeout-method thread -k "random_sweep" > gpurun_out/fuzz_sweep_big.log 2>&1
rc=$?
tail -3 gpurun_out/fuzz_sweep_big.log
exit $rc
