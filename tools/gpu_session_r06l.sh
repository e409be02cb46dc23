# Round-6 session l: tile sizes of the tiled pack (units / 8 / 4 KiB) and of
# the whole-word unpack (4 / 8 / 16 KiB), interleaved twice.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in a b c; do
    case $v in
      a) E="MVX_PACK_TILES=0 MVX_UNPACK_TILE_KIB=4";;
      b) E="MVX_PACK_TILE_KIB=8 MVX_UNPACK_TILE_KIB=8";;
      c) E="MVX_PACK_TILE_KIB=4 MVX_UNPACK_TILE_KIB=16";;
    esac
    env $E timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06l_${v}_$r.jsonl 2>> gpurun_out/r06l.err || { tail -20 gpurun_out/r06l.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for r in (1, 2):
    rows = {v: [json.loads(l) for l in open("gpurun_out/r06l_%s_%d.jsonl" % (v, r))] for v in "abc"}
    for i, a in enumerate(rows["a"]):
        lab = ("units", "tiles8", "tiles4") if a["dir"] == "pack" else ("merge4", "merge8", "merge16")
        print(r, "%-44s %-6s %s %7.2f  %s %7.2f  %s %7.2f" % (a["type"][:44], a["dir"], lab[0], a["us"], lab[1], rows["b"][i]["us"], lab[2], rows["c"][i]["us"]))
PY
