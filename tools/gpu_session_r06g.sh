# Round-6 session g: the slice schedule with kinds mixed within ranks, the
# rccl-net random suites, and a 600-case random sweep per world size.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 500 --timeout-method thread \
  tests/test_gpu_multiproc.py -k "slice or net_transport" > gpurun_out/r06g_mp.log 2>&1 || { tail -60 gpurun_out/r06g_mp.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" gpurun_out/r06g_mp.log; tail -1 gpurun_out/r06g_mp.log
MVX_MP_CASES=600 timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 500 --timeout-method thread \
  tests/test_gpu_multiproc.py -k "random_host" > gpurun_out/r06g_random600.log 2>&1 || { tail -60 gpurun_out/r06g_random600.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" gpurun_out/r06g_random600.log; tail -1 gpurun_out/r06g_random600.log
