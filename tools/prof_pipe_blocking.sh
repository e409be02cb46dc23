# PIPE through the blocking MPI_Allreduce (the null stream, as the MPI entry
# points issue it) at p = 2 over rccl-net: device buffers on both ranks,
# 48 MiB per rank (under MVX_SLICE_MIN_MIB, so the exchange variant, not the
# slice schedule, runs), a kernel trace of each rank, then tools/overlap.py
# on rank 0's -- how much of the combine time ran while an RCCL kernel was
# in flight on another queue.  P2P beside it as the no-overlap reference.
# The null-stream PIPE call forks to the communicator's non-blocking stream
# (csrc/mvx_exec.c run_device_pipe): without that, the legacy null stream
# would wait for the blocking combine stream between slices.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=2
for ex in ${EXCHS:-p2p pipe}; do
  port=$((29900 + ${#ex}))
  pids=""
  for r in 0 1; do
    rm -rf gpurun_out/prof_pb_${ex}_r$r
    MVX_EXCHANGE=$ex MASTER_PORT=$port RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace \
      --output-format csv -d gpurun_out/prof_pb_${ex}_r$r -o r$r -- \
      python3 tools/host_multi.py --mib ${MIB:-48} --kinds device --reps ${REPS:-8} \
      > gpurun_out/prof_pb_${ex}_r$r.log 2>&1 &
    pids="$pids $!"
  done
  for p in $pids; do wait $p || exit 1; done
  grep -h '^{' gpurun_out/prof_pb_${ex}_r0.log gpurun_out/prof_pb_${ex}_r1.log || exit 1
  f=$(find gpurun_out/prof_pb_${ex}_r0 -name "*kernel_trace.csv" | head -1)
  [ -n "$f" ] || exit 1
  python3 tools/overlap.py "$f" "$ex blocking MPI_Allreduce (null stream)" || exit 1
done
