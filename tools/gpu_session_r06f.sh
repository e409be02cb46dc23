# Round-6 session f: the multi-process suites with buffer kinds mixed within
# a rank too (mixed / random / sliced, host transport and rccl-net).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_multiproc.py -k "mixed or random or sliced" > gpurun_out/r06f_mp.log 2>&1 || { tail -60 gpurun_out/r06f_mp.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" gpurun_out/r06f_mp.log; tail -1 gpurun_out/r06f_mp.log
