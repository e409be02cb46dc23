# Round-5 measurement session: the Python graph-eviction test, PIPE through
# the blocking MPI_Allreduce (null stream) traced, then the N = 1 headline:
# PMC passes (FETCH / WRITE), the driver's command under the kernel trace,
# the combine kernels' PMC passes, and the driver's own bench command.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread "tests/test_gpu_multiproc.py::test_graphs_rccl_net_evicting" > gpurun_out/r05_graph_fix2.log 2>&1 || exit 1
bash tools/prof_pipe_blocking.sh > gpurun_out/r05_pipe_blocking.log 2>&1 || exit 1
bash tools/gpu_round.sh pmc > gpurun_out/r05_round_pmc.log 2>&1 || exit 1
bash tools/gpu_round.sh prof > gpurun_out/r05_round_prof.log 2>&1 || exit 1
bash tools/gpu_round.sh pmc_kernels > gpurun_out/r05_round_pmck.log 2>&1 || exit 1
bash tools/gpu_round.sh bench > gpurun_out/r05_round_bench.log 2>&1 || exit 1
