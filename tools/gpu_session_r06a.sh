# Round-6 first session: the new shim / registration / graph-cache / merge
# unpack tests, the contradicted-hint and graph rccl-net suites, and the pack
# kernels with and without whole-word unpack.  Every GPU step has its own
# limit; the chain stops at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
: skip timeout -k 10 300 $PT tests/test_gpu_types.py -k whole_word > gpurun_out/r06a_merge_test.log 2>&1 || { tail -40 gpurun_out/r06a_merge_test.log; exit 1; }
tail -2 gpurun_out/r06a_merge_test.log
timeout -k 10 500 $PT -s tests/test_gpu_integration.py tests/test_gpu_host_register.py > gpurun_out/r06a_shim_reg.log 2>&1 || { tail -60 gpurun_out/r06a_shim_reg.log; exit 1; }
grep -h "median us" gpurun_out/r06a_shim_reg.log; tail -2 gpurun_out/r06a_shim_reg.log
timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06a_pack_merge.jsonl 2> gpurun_out/r06a_pack_merge.err || { tail -20 gpurun_out/r06a_pack_merge.err; exit 1; }
MVX_UNPACK_MERGE=0 timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06a_pack_masked.jsonl 2> gpurun_out/r06a_pack_masked.err || { tail -20 gpurun_out/r06a_pack_masked.err; exit 1; }
grep unpack gpurun_out/r06a_pack_merge.jsonl gpurun_out/r06a_pack_masked.jsonl | cut -c1-330
timeout -k 10 600 $PT tests/test_gpu_multiproc.py -k "sliced or graph" > gpurun_out/r06a_mp.log 2>&1 || { tail -60 gpurun_out/r06a_mp.log; exit 1; }
tail -3 gpurun_out/r06a_mp.log
