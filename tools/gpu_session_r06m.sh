# Round-6 session m: the final pack / unpack build -- derived-type parity,
# the pack kernels (tiled pack and whole-word unpack on, then both off), and
# their HBM bytes (PMC, one counter per pass).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_types.py tests/test_gpu_derived.py tests/test_gpu_integration.py -k "not latency" > gpurun_out/r06m_types.log 2>&1 || { tail -40 gpurun_out/r06m_types.log; exit 1; }
tail -1 gpurun_out/r06m_types.log
timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06m_pack_on.jsonl 2> gpurun_out/r06m_pack_on.err || { tail -20 gpurun_out/r06m_pack_on.err; exit 1; }
MVX_PACK_TILES=0 MVX_UNPACK_MERGE=0 timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06m_pack_off.jsonl 2> gpurun_out/r06m_pack_off.err || { tail -20 gpurun_out/r06m_pack_off.err; exit 1; }
python3 - <<'PY'
import json
m = [json.loads(l) for l in open("gpurun_out/r06m_pack_on.jsonl")]
k = [json.loads(l) for l in open("gpurun_out/r06m_pack_off.jsonl")]
for a, b in zip(m, k):
    print("%-48s %-6s on %7.2f us  off %7.2f us" % (a["type"], a["dir"], a["us"], b["us"]))
PY
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/r06m_pmc_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r06m_pmc_$c -o p -- python3 tools/bench_pack.py \
    > gpurun_out/r06m_pmc_$c.log 2>&1 || { tail -20 gpurun_out/r06m_pmc_$c.log; exit 1; }
done
python3 tools/pmc_pack_summary.py gpurun_out/r06m_pmc_FETCH_SIZE gpurun_out/r06m_pmc_WRITE_SIZE gpurun_out/r06m_pack_on.jsonl > gpurun_out/r06m_pmc_pack.txt || exit 1
cut -c1-160 gpurun_out/r06m_pmc_pack.txt
