# How often does capture -> instantiate -> launch -> hipGraphExecDestroy of a
# fork / join graph crash, per HIP runtime?  Each line of the probe is a
# fresh pair of processes; a hung or crashed pair is reported, the next runs.
cd $GRAFT_REPO_ROOT
for rep in 1 2 3 4; do
  for bin in graph_probe2_70 graph_probe2; do
    timeout -k 10 150 tools/$bin churn_fork_norccl churn_single churn_fork_keep 2>/dev/null | sed "s/^/$bin rep $rep: /"
  done
done
