# Round-6 session k: tiled pack tile size A/B (8 vs 16 KiB) against the unit
# kernel, interleaved twice.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in u16 t8 t4; do
    case $v in u16) E="MVX_PACK_TILES=0";; t4) E="MVX_PACK_TILE_KIB=4";; t8) E="MVX_PACK_TILE_KIB=8";; esac
    env $E timeout -k 10 240 python3 tools/bench_pack.py > gpurun_out/r06k_${v}_$r.jsonl 2>> gpurun_out/r06k.err || { tail -20 gpurun_out/r06k.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for r in (1, 2):
    rows = {v: [json.loads(l) for l in open("gpurun_out/r06k_%s_%d.jsonl" % (v, r))] for v in ("u16", "t8", "t4")}
    for i, a in enumerate(rows["u16"]):
        if a["dir"] == "pack":
            print(r, "%-48s units %7.2f  tiles8 %7.2f  tiles4 %7.2f" % (a["type"], a["us"], rows["t8"][i]["us"], rows["t4"][i]["us"]))
PY
