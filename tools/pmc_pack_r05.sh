# HBM bytes of the pack / unpack kernels (rocprofv3 PMC, one counter per
# pass): FETCH_SIZE (doubled on gfx950, MI355X_MICROARCH.md) and WRITE_SIZE
# per dispatch of k_pack_units, over tools/bench_pack.py.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_pack_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_pack_$c -o p -- python3 tools/bench_pack.py \
    > gpurun_out/pmc_pack_$c.log 2>&1 || { tail -20 gpurun_out/pmc_pack_$c.log; exit 1; }
done
find gpurun_out/pmc_pack_FETCH_SIZE gpurun_out/pmc_pack_WRITE_SIZE -name "*counter_collection.csv"
