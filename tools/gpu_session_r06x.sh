# Round-6 session x: the final build end to end -- smoke, the whole GPU
# suite, the driver's bench command, its kernel trace and the C2 PMC bytes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round.sh smoke && bash tools/gpu_round.sh test && bash tools/gpu_round.sh bench && \
  bash tools/gpu_round.sh prof && bash tools/gpu_round.sh pmc
