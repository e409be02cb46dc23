# Round-6 session d: the driver's bench command under the kernel trace and
# bare, smoke, and the C2 kernel's HBM bytes (PMC, one counter per pass).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round.sh prof > gpurun_out/r06d_prof.log 2>&1 || { tail -30 gpurun_out/r06d_prof.log; exit 1; }
bash tools/gpu_round.sh bench > gpurun_out/r06d_bench.log 2>&1 || { tail -30 gpurun_out/r06d_bench.log; exit 1; }
cut -c1-600 gpurun_out/bench.json
bash tools/gpu_round.sh smoke > gpurun_out/r06d_smoke.log 2>&1 || { tail -30 gpurun_out/r06d_smoke.log; exit 1; }
tail -2 gpurun_out/r06d_smoke.log
bash tools/gpu_round.sh pmc > gpurun_out/r06d_pmc.log 2>&1 || { tail -30 gpurun_out/r06d_pmc.log; exit 1; }
cat gpurun_out/pmc_c2.json
