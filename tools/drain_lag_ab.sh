# A/B of the host op pipeline's drain lag (csrc/mvx_hostop.c,
# MVX_HOST_DRAIN_LAG): pageable MPIR_SUM float32 at 64 / 256 MiB, lag 1
# (rounds 1-4) and 2, interleaved, three passes each.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/drain_lag_ab.jsonl
: > $out
for pass in 1 2 3; do
  for lag in 1 2; do
    MVX_HOST_DRAIN_LAG=$lag timeout -k 10 120 python3 tools/bench_host.py --min-mib 64 --cases op_pageable,ar1_pageable \
      > gpurun_out/dl.tmp 2>&1 || { cat gpurun_out/dl.tmp; exit 1; }
    grep '^{' gpurun_out/dl.tmp | sed "s/^{/{\"lag\": $lag, \"pass\": $pass, /" >> $out
  done
done
cat $out
