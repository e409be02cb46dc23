# Round-6 session c: the whole GPU suite on the round's build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round.sh test > gpurun_out/r06c_test.log 2>&1 || { tail -40 gpurun_out/r06c_test.log; exit 1; }
tail -3 gpurun_out/r06c_test.log
