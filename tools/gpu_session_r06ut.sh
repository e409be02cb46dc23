# Round-6 session ut: the whole-word unpack reading the chunk table for 1-
# and 2-byte units: parity (types, derived, random maps, host register) and
# the pack bench, table on / off interleaved (tab=1 / tab=0:
# MVX_UNPACK_CHUNK_TAB).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_types.py tests/test_gpu_derived.py tests/test_gpu_host_register.py > gpurun_out/r06ut_pytest.log 2>&1 || { tail -40 gpurun_out/r06ut_pytest.log; exit 1; }
tail -2 gpurun_out/r06ut_pytest.log
rm -f gpurun_out/r06ut_tab.txt
for tab in 1 0 1 0; do
  MVX_UNPACK_CHUNK_TAB=$tab timeout -k 10 300 python3 tools/bench_pack.py > gpurun_out/r06ut_pack_tab$tab.jsonl 2> gpurun_out/r06ut_pack.err || { tail -20 gpurun_out/r06ut_pack.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r06ut_pack_tab$tab.jsonl'):
    d = json.loads(l)
    print(d['dir'], end=' '); print('tab=$tab', d['type'][:40], d['us'])" >> gpurun_out/r06ut_tab.txt
done
cat gpurun_out/r06ut_tab.txt
