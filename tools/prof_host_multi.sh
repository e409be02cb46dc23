# Host buffers at p = 2 over rccl-net (two ranks sharing the GPU, RCCL's
# socket transport): rank 0 host buffers, rank 1 device buffers (KINDS), a
# 256 MiB MPI_Allreduce(SUM, float32); each rank under rocprofv3 with kernel
# and memory-copy traces; then tools/host_overlap.py on rank 0's (the host
# rank): how much its H2D, D2H and the collective overlap.  Run once with the
# slice schedule (default) and once with it off (MVX_SLICE_MIN_MIB=65536:
# HBM mirrors, the round-4 default).  Rates are socket-bound here.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=2
MIB=${MIB:-256}
for mode in ${MODES:-sliced mirrors}; do
  if [ $mode = mirrors ]; then export MVX_SLICE_MIN_MIB=65536; else unset MVX_SLICE_MIN_MIB; fi
  port=$((29800 + ${#mode}))
  pids=""
  for r in 0 1; do
    rm -rf gpurun_out/prof_host_${mode}_r$r
    MASTER_PORT=$port RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace \
      --output-format csv -d gpurun_out/prof_host_${mode}_r$r -o r$r -- \
      python3 tools/host_multi.py --mib $MIB --kinds ${KINDS:-host,device} --reps ${REPS:-4} \
      > gpurun_out/prof_host_${mode}_r$r.log 2>&1 &
    pids="$pids $!"
  done
  for p in $pids; do wait $p || exit 1; done
  grep -h '^{' gpurun_out/prof_host_${mode}_r0.log gpurun_out/prof_host_${mode}_r1.log || exit 1
  python3 tools/host_overlap.py gpurun_out/prof_host_${mode}_r0 "$mode rank 0 (${KINDS:-host,device})" || exit 1
done
