# Round-6 session h: graph tests after the graph-cache changes, then fresh
# seeded sweeps on the round's build (3000 collective cases, 1000 op-function
# cases).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
  tests/test_gpu_graph_app.py tests/test_gpu_multiproc.py tests/test_gpu_exec.py -k "graph" > gpurun_out/r06h_graphs.log 2>&1 || { tail -60 gpurun_out/r06h_graphs.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" gpurun_out/r06h_graphs.log | cut -c1-120; tail -1 gpurun_out/r06h_graphs.log
SEED=6060606 bash tools/fuzz_sweep_big_r05.sh || exit 1
cp gpurun_out/fuzz_sweep_big.log gpurun_out/r06h_fuzz_sweep_3000_seed6060606.log
SEED=6161616 bash tools/fuzz_ops_big_r05.sh || exit 1
cp gpurun_out/fuzz_ops_big.log gpurun_out/r06h_fuzz_ops_1000_seed6161616.log
