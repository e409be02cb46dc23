# Round-6 session u: the unit kernel with global (not flat) stores: parity
# of the derived-type suites and the pack bench with the tile kernels on and
# off (off = the unit kernel everywhere it applies).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_types.py tests/test_gpu_derived.py > gpurun_out/r06u_pytest.log 2>&1 || { tail -30 gpurun_out/r06u_pytest.log; exit 1; }
tail -2 gpurun_out/r06u_pytest.log
timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/r06u_pack_on.jsonl 2> gpurun_out/r06u_pack_on.err || { tail -20 gpurun_out/r06u_pack_on.err; exit 1; }
MVX_PACK_TILES=0 MVX_UNPACK_MERGE=0 timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/r06u_pack_off.jsonl 2> gpurun_out/r06u_pack_off.err || { tail -20 gpurun_out/r06u_pack_off.err; exit 1; }
echo done
