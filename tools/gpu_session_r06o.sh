# Round-6 session o: tile kernels over 2- and 1-byte units -- parity, then
# the pack kernels with the tile kernels on and off.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_types.py tests/test_gpu_derived.py > gpurun_out/r06o_types.log 2>&1 || { tail -40 gpurun_out/r06o_types.log; exit 1; }
tail -1 gpurun_out/r06o_types.log
timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/r06o_pack_on.jsonl 2> gpurun_out/r06o_pack_on.err || { tail -20 gpurun_out/r06o_pack_on.err; exit 1; }
MVX_PACK_TILES=0 MVX_UNPACK_MERGE=0 timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/r06o_pack_off.jsonl 2> gpurun_out/r06o_pack_off.err || { tail -20 gpurun_out/r06o_pack_off.err; exit 1; }
python3 - <<'PY'
import json
m = [json.loads(l) for l in open("gpurun_out/r06o_pack_on.jsonl")]
k = [json.loads(l) for l in open("gpurun_out/r06o_pack_off.jsonl")]
for a, b in zip(m, k):
    print("%-48s %-6s on %7.2f us  off %7.2f us  line_frac %.3f / %.3f" % (a["type"], a["dir"], a["us"], b["us"], a["line_frac"], b["line_frac"]))
PY
