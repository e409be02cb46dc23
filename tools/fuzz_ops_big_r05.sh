# One-off seeded sweep of the op functions on random operand kinds (HBM,
# pageable, page-locked; offset by an element) after the round-5 host-path
# changes (zero copy for page-locked operands, drain lag 2): 40 batches x 25
# cases, a fresh seed, against the oracle.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MVX_FUZZ_OP_BATCHES=40 MVX_FUZZ_SEED=${SEED:-5050505} timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "random_op_functions" > gpurun_out/fuzz_ops_big.log 2>&1
rc=$?
tail -3 gpurun_out/fuzz_ops_big.log
exit $rc
