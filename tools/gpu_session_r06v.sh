# Round-6 session v: random type maps through every pack / unpack kernel,
# then the tile sizes again on the flat-free kernels (8 vs 16 KiB).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_types.py -k "random_type_maps" > gpurun_out/r06v_pytest.log 2>&1 || { tail -40 gpurun_out/r06v_pytest.log; exit 1; }
tail -2 gpurun_out/r06v_pytest.log
for kib in 8 16 8 16; do
  MVX_PACK_TILE_KIB=$kib MVX_UNPACK_TILE_KIB=$kib timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/r06v_pack_tile$kib.jsonl 2> gpurun_out/r06v_pack.err || { tail -20 gpurun_out/r06v_pack.err; exit 1; }
  cat gpurun_out/r06v_pack_tile$kib.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$kib', d['type'][:28], d['dir'], d['us'])" >> gpurun_out/r06v_tiles.txt
done
cat gpurun_out/r06v_tiles.txt
