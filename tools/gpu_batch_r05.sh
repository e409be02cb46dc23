set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread "tests/test_gpu_multiproc.py::test_slice_schedule_any_kinds" "tests/test_gpu_multiproc.py::test_mixed_buffer_kinds_across_ranks" "tests/test_gpu_exec.py::test_pipelined_exchange_matches_reference" > gpurun_out/r05_batch2_tests.log 2>&1 || exit 1
MODES="sliced mirrors" bash tools/prof_host_multi.sh > gpurun_out/r05_prof_host_multi.log 2>&1 || exit 1
echo probes > gpurun_out/r05_probe.log
timeout -k 10 300 tools/graph_probe2 >> gpurun_out/r05_probe.log 2>&1
echo "rc $?" >> gpurun_out/r05_probe.log
