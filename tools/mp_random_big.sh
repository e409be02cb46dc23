cd $GRAFT_REPO_ROOT
export MVX_MP_CASES=500
timeout -k 10 800 python -u -m pytest tests/test_gpu_multiproc.py -m gpu -x -q -p no:cacheprovider --timeout 700 --timeout-method thread -k "random" > gpurun_out/t_mp_big.log 2>&1
rc=$?
grep -E "^E |passed|failed" gpurun_out/t_mp_big.log | head
exit $rc
