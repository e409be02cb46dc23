# Round-6 session b: whole-word unpack with 16-byte packed reads -- the
# derived-type parity suites, the pack kernels with and without it, their
# HBM bytes (PMC, one counter per pass), and the route agreement's latency.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_types.py tests/test_gpu_derived.py > gpurun_out/r06b_types.log 2>&1 || { tail -40 gpurun_out/r06b_types.log; exit 1; }
tail -1 gpurun_out/r06b_types.log
timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06b_pack_merge.jsonl 2> gpurun_out/r06b_pack_merge.err || { tail -20 gpurun_out/r06b_pack_merge.err; exit 1; }
MVX_UNPACK_MERGE=0 timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06b_pack_masked.jsonl 2> gpurun_out/r06b_pack_masked.err || { tail -20 gpurun_out/r06b_pack_masked.err; exit 1; }
python3 - <<'PY'
import json
m = [json.loads(l) for l in open("gpurun_out/r06b_pack_merge.jsonl")]
k = [json.loads(l) for l in open("gpurun_out/r06b_pack_masked.jsonl")]
for a, b in zip(m, k):
    if a["dir"] == "unpack":
        print("%-48s merge %7.2f us  masked %7.2f us  rmw_frac %.3f / %.3f" % (a["type"], a["us"], b["us"], a["rmw_frac"], b["rmw_frac"]))
PY
timeout -k 10 200 $PT -s tests/test_gpu_integration.py -k latency > gpurun_out/r06b_latency.log 2>&1 || { tail -30 gpurun_out/r06b_latency.log; exit 1; }
grep -h "median us" gpurun_out/r06b_latency.log
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/r06b_pmc_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r06b_pmc_$c -o p -- python3 tools/bench_pack.py \
    > gpurun_out/r06b_pmc_$c.log 2>&1 || { tail -20 gpurun_out/r06b_pmc_$c.log; exit 1; }
done
find gpurun_out/r06b_pmc_FETCH_SIZE gpurun_out/r06b_pmc_WRITE_SIZE -name "*counter_collection.csv"
