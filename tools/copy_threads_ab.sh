# Copy-pool size A/B after the drain-lag change: MVX_COPY_THREADS 8 / 12 / 16
# on the pageable op and p = 1 Allreduce (64 / 256 MiB), interleaved, two
# passes (tools/bench_host.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/copy_threads_ab.jsonl; : > $out
for pass in 1 2; do for nt in 8 12 16; do
  MVX_COPY_THREADS=$nt timeout -k 10 120 python3 tools/bench_host.py --min-mib 64 --cases op_pageable,ar1_pageable \
    > gpurun_out/ct.tmp 2>&1 || { cat gpurun_out/ct.tmp; exit 1; }
  grep '^{' gpurun_out/ct.tmp | sed "s/^{/{\"threads\": $nt, \"pass\": $pass, /" >> $out
done; done
cat $out
