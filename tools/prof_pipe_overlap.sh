# PIPE against P2P at p = 2 over rccl-net (C3 shapes, 64 MiB per rank): a
# kernel trace of each rank, then tools/overlap.py on rank 0's -- how much of
# the combine time ran while an RCCL kernel was in flight on the other stream.
# EXCHS="pipe" MVX_PIPE_STREAM=plain|priority|cumask for the stream A/B.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=2
for ex in ${EXCHS:-p2p pipe}; do
  rm -rf gpurun_out/prof_ov_${ex}_r0 gpurun_out/prof_ov_${ex}_r1
  port=$((29700 + ${#ex}))
  for r in 0 1; do
    MASTER_PORT=$port RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ov_${ex}_r$r -o r$r -- python3 bench.py --gpus 2 --transport rccl-net --config c3 --mib 64 --steps 10 --warmup 3 --tune-steps 2 --exchange $ex --no-native --extra-configs none > gpurun_out/prof_ov_${ex}_r$r.log 2>&1 &
  done
  wait || exit 1
  f=$(find gpurun_out/prof_ov_${ex}_r0 -name "*kernel_trace.csv" | head -1)
  [ -n "$f" ] || exit 1
  python3 tools/overlap.py "$f" "$ex ${MVX_PIPE_STREAM:-default}" || exit 1
done
