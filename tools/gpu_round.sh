#!/bin/bash
# One GPU-box session, by stage: smoke, tests, bench, PMC passes, kernel
# trace, kernel micro-benches, host-buffer rates.  Every GPU step has its own
# time limit; the chain stops at the first failure (no retries).
#   tools/gpu_round.sh STAGE [pytest args]   (STAGE: all smoke test bench pmc prof kernels host
#   bench_ab kernels_ab pmc_kernels rccl_net overlap)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
shift || true
run() { echo "== $*" ; "$@"; }
ok=0
if [[ $STAGE == all || $STAGE == smoke ]]; then
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == test ]]; then
  run timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  # the driver's own command
  run timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STAGE == all || $STAGE == pmc ]]; then
  # one counter set per pass (FETCH_SIZE takes 3 TCC counters, WRITE_SIZE 2)
  rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
  run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernels > gpurun_out/pmc_fetch.log 2>&1 || { tail -30 gpurun_out/pmc_fetch.log; exit 1; }
  run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernels > gpurun_out/pmc_write.log 2>&1 || { tail -30 gpurun_out/pmc_write.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write "k_combine<2, float, 2, 4, 1, 0>" sum_f32_k2_nt 268435456 805306368 gpurun_out/pmc_c2.json || exit 1
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  rm -rf gpurun_out/prof_kt
  # the driver's own command under the kernel trace; every dispatch of the
  # C2 kernel in order (prewarm / warmup / timed / evented / parity)
  run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_kt.log 2>&1 || { tail -30 gpurun_out/prof_kt.log; exit 1; }
  find gpurun_out/prof_kt -name "*stats*"
  python3 tools/dispatch_series.py gpurun_out/prof_kt "k_combine<2, float, 2, 4, 1, 0>" 20 gpurun_out/dispatch_series.json || exit 1
fi
if [[ $STAGE == all || $STAGE == kernels ]]; then
  run timeout -k 10 300 python tools/bench_kernels.py "$@" > gpurun_out/bench_kernels.jsonl 2> gpurun_out/bench_kernels.err || { tail -20 gpurun_out/bench_kernels.err; exit 1; }
  cat gpurun_out/bench_kernels.jsonl
fi
if [[ $STAGE == all || $STAGE == host ]]; then
  run timeout -k 10 300 python tools/bench_host.py "$@" > gpurun_out/bench_host.jsonl 2> gpurun_out/bench_host.err || { tail -20 gpurun_out/bench_host.err; exit 1; }
  cat gpurun_out/bench_host.jsonl
fi
if [[ $STAGE == bench_ab ]]; then
  # the driver's command with and without the prewarm, interleaved
  for r in 1 2; do
    for pw in 0 300; do
      run timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --prewarm-ms $pw --no-kernels > gpurun_out/bench_pw${pw}_$r.json 2>> gpurun_out/bench_ab.err || exit 1
      cut -c1-400 gpurun_out/bench_pw${pw}_$r.json
    done
  done
fi
if [[ $STAGE == kernels_ab ]]; then
  # fixed-tree programs (default) against the generic masked program
  # (MVX_PROG_GENERIC=1), interleaved on one box
  for r in 1 2; do
    for g in 0 1; do
      MVX_PROG_GENERIC=$g run timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels_g${g}_$r.jsonl 2>> gpurun_out/bench_kernels.err || exit 1
    done
  done
  for f in gpurun_out/bench_kernels_g*_*.jsonl; do echo "-- $f"; cut -c1-150 $f; done
fi
if [[ $STAGE == pmc_kernels ]]; then
  rm -rf gpurun_out/pmck_f gpurun_out/pmck_w
  run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmck_f -o f -- python3 tools/bench_kernels.py > gpurun_out/pmck_f.log 2>&1 || exit 1
  run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmck_w -o w -- python3 tools/bench_kernels.py > gpurun_out/pmck_w.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmck_f gpurun_out/pmck_w "k_tree_body<2, float, 8, 2>" sum_f32_k8_nt 33554432 301989888 gpurun_out/pmc_c3.json && \
  python3 tools/pmc_summary.py gpurun_out/pmck_f gpurun_out/pmck_w "k_chain_body<5, unsigned long, 4, 2>" band_u64_k4_nt 268435456 1342177280 gpurun_out/pmc_c4.json && \
  python3 tools/pmc_summary.py gpurun_out/pmck_f gpurun_out/pmck_w "k_tree_body<11, mvx::pfi, 8, 2>" maxloc_float_int_k8_nt 67108864 603979776 gpurun_out/pmc_c5.json || exit 1
fi
if [[ $STAGE == rccl_net ]]; then
  # RCCL communicators whose ranks share the one GPU (NCCL_HOSTID per rank,
  # RCCL's socket transport): the full-size bench legs and random sweeps
  TRANSPORT=rccl-net tools/rehearse_full.sh c3 c4 || exit 1
  MVX_MP_CASES=${MVX_MP_CASES:-300} tools/rccl_net_sweep.sh > gpurun_out/rccl_net_sweep.jsonl || { cat gpurun_out/rccl_net_sweep.jsonl; exit 1; }
  cat gpurun_out/rccl_net_sweep.jsonl
fi
if [[ $STAGE == overlap ]]; then
  # PIPE's combines under RCCL's transfers (kernel traces, p = 2 over rccl-net)
  bash tools/prof_pipe_overlap.sh > gpurun_out/overlap.jsonl 2> gpurun_out/overlap.err || { tail -20 gpurun_out/overlap.err; exit 1; }
  cat gpurun_out/overlap.jsonl
fi
