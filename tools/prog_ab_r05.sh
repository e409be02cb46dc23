# The masked-program kernels (k = 3, 5, 6, 7) under U = 2 and residency caps (A/B, tools/bench_kernels.py ks)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "X=0" "MVX_PROG_U=2" "MVX_CAP_PROG=4" "MVX_CAP_PROG=3" "MVX_CAP_PROG=2"; do
  env $cfg timeout -k 10 200 python3 tools/bench_kernels.py ks 2>/dev/null | grep -E '"K-(102-10|105-8)-(tree|chain)-k(3|5|6|7)"' | sed "s/^{/{\"cfg\": \"$cfg\", /" >> gpurun_out/k3_ab.jsonl || exit 1
done
