# Round-6 session z: the registered op path against the pinned one on one
# box, zero copy on / off, two interleaved passes (256 MiB and 128 MiB).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r06z_zc_ab.jsonl; : > $out
for pass in 1 2; do for zc in 0 1; do
  MVX_HOST_ZEROCOPY=$zc timeout -k 10 180 python3 tools/bench_host.py --min-mib 128 --cases op_pinned,op_registered \
    > gpurun_out/zc.tmp 2>&1 || { cat gpurun_out/zc.tmp; exit 1; }
  grep '^{' gpurun_out/zc.tmp | sed "s/^{/{\"zerocopy\": $zc, \"pass\": $pass, /" >> $out
done; done
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); print(d['zerocopy'], d['pass'], d['case'], d['bytes'] >> 20, d['us'], d.get('registered'))"
