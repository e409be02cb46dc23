# Round-5 late-build session (SWAR 1-byte ops, pair apply body, unit pack kernels, 4-leaf programs) on a fresh box: the driver's bench command
# under the kernel trace and bare (before anything warms the GPU), smoke,
# then the whole GPU suite.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round.sh prof > gpurun_out/r05f_prof.log 2>&1 || exit 1
bash tools/gpu_round.sh bench > gpurun_out/r05f_bench.log 2>&1 || exit 1
bash tools/gpu_round.sh smoke > gpurun_out/r05f_smoke.log 2>&1 || exit 1
bash tools/gpu_round.sh test > gpurun_out/r05f_test.log 2>&1 || exit 1
