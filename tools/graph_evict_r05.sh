# Round-5 reproduction of the round-4 hipGraphLaunch SIGSEGV with graphs
# destroyed mid-life again (MVX_GRAPH_EVICT=1, one graph per communicator):
# the C application (tools/graph_app.c) on the image's ROCm and on torch's
# bundled runtime, then the Python suite's graph job list at p = 2 with a
# native backtrace on a crash (tools/segv_bt.c).  Each step is bounded; the
# crash is a host-side SIGSEGV in the launching process.
cd $GRAFT_REPO_ROOT
export MVX_GRAPH_TRACE=1
MVX_GRAPH_EVICT=1 MVX_GRAPH_CACHE=1 timeout -k 10 120 tools/graph_app > gpurun_out/r05_graph_app_evict72.log 2>&1
echo "rc $?" >> gpurun_out/r05_graph_app_evict72.log
MVX_GRAPH_EVICT=1 MVX_GRAPH_CACHE=1 timeout -k 10 120 tools/graph_app70 > gpurun_out/r05_graph_app_evict70.log 2>&1
echo "rc $?" >> gpurun_out/r05_graph_app_evict70.log
AMD_LOG_LEVEL=1 MVX_MP_TRACE=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread "tests/test_gpu_multiproc.py::test_graphs_rccl_net_evicting[2]" > gpurun_out/r05_graph_evict2.log 2>&1
echo "rc $?" >> gpurun_out/r05_graph_evict2.log
timeout -k 10 200 tools/graph_probe2 copy_then_pipe null_copy_then_pipe > gpurun_out/r05_probe72d.log 2>&1
echo "rc $?" >> gpurun_out/r05_probe72d.log
timeout -k 10 200 tools/graph_probe2_70 copy_then_pipe null_copy_then_pipe > gpurun_out/r05_probe70d.log 2>&1
echo "rc $?" >> gpurun_out/r05_probe70d.log
AMD_LOG_LEVEL=1 timeout -k 10 240 tools/graph_probe2_70 churn_pipe churn_fork_norccl churn_p2p > gpurun_out/r05_probe70e.log 2>&1
echo "rc $?" >> gpurun_out/r05_probe70e.log
AMD_LOG_LEVEL=1 timeout -k 10 240 tools/graph_probe2 churn_pipe churn_fork_norccl churn_p2p > gpurun_out/r05_probe72e.log 2>&1
echo "rc $?" >> gpurun_out/r05_probe72e.log
