# Round-6 session n: where the 8 leaves of the C3 combine sit (slot stagger)
# against the current body kernel, two passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 tools/tune_combine_layout.py fine > gpurun_out/r06n_layout_$r.jsonl 2> gpurun_out/r06n.err || { tail -20 gpurun_out/r06n.err; exit 1; }
done
paste -d' ' <(cut -c1-80 gpurun_out/r06n_layout_1.jsonl) <(cut -d, -f3 gpurun_out/r06n_layout_2.jsonl)
