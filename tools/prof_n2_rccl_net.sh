cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29655 WORLD_SIZE=2
rm -rf gpurun_out/prof_n2_r0 gpurun_out/prof_n2_r1
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_n2_r$r -o r$r -- python3 bench.py --gpus 2 --transport rccl-net --config c3 --steps 20 --warmup 5 --tune-steps 2 --exchange p2p > gpurun_out/prof_n2_r$r.log 2>&1 &
done
wait
grep '"metric"' gpurun_out/prof_n2_r0.log | cut -c1-300
find gpurun_out/prof_n2_r0 -name "*kernel_stats*" -exec head -8 {} \;
