# Round-6 session t: the tile kernels without flat accesses (unit offsets
# from LDS as a template argument, trash-word stores, byte-stored hull
# edges): parity of the derived-type suites, the pack bench, and HBM bytes
# (PMC, one counter per pass).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_types.py tests/test_gpu_derived.py > gpurun_out/r06t_pytest.log 2>&1 || { tail -30 gpurun_out/r06t_pytest.log; exit 1; }
tail -2 gpurun_out/r06t_pytest.log
timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/r06t_pack_on.jsonl 2> gpurun_out/r06t_pack_on.err || { tail -20 gpurun_out/r06t_pack_on.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/r06t_pmc_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r06t_pmc_$c -o p -- python3 tools/bench_pack.py \
    > gpurun_out/r06t_pmc_$c.log 2>&1 || { tail -20 gpurun_out/r06t_pmc_$c.log; exit 1; }
done
python3 tools/pmc_pack_summary.py gpurun_out/r06t_pmc_FETCH_SIZE gpurun_out/r06t_pmc_WRITE_SIZE gpurun_out/r06t_pack_on.jsonl > gpurun_out/r06t_pmc_pack.txt || exit 1
cut -c1-175 gpurun_out/r06t_pmc_pack.txt
