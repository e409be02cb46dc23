#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, 1-GPU bench, rocprof trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
run() { echo "== $*" ; "$@"; }
if [[ $STAGE == all || $STAGE == smoke ]]; then
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == test ]]; then
  run timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  run timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STAGE == all || $STAGE == pmc ]]; then
  rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
  run timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || { tail -30 gpurun_out/pmc_fetch.log; exit 1; }
  run timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || { tail -30 gpurun_out/pmc_write.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write "k_combine<2, float, 2, 1, 4, 1>" sum_f32_k2_nt 268435456 805306368 gpurun_out/pmc_c2.json
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 || { tail -30 gpurun_out/prof_kt.log; exit 1; }
  find gpurun_out/prof_kt -name "*stats*" | head
fi
if [[ $STAGE == all || $STAGE == kernels ]]; then
  run timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels.jsonl 2> gpurun_out/bench_kernels.err || { tail -20 gpurun_out/bench_kernels.err; exit 1; }
  cat gpurun_out/bench_kernels.jsonl
fi
if [[ $STAGE == all || $STAGE == host ]]; then
  run timeout -k 10 300 python tools/bench_host.py > gpurun_out/bench_host.jsonl 2> gpurun_out/bench_host.err || { tail -20 gpurun_out/bench_host.err; exit 1; }
  cat gpurun_out/bench_host.jsonl
fi
if [[ $STAGE == x87 ]]; then
  run timeout -k 10 300 python tools/bench_kernels.py x87 > gpurun_out/bench_kernels_x87.jsonl 2> gpurun_out/bench_kernels.err || { tail -20 gpurun_out/bench_kernels.err; exit 1; }
  cat gpurun_out/bench_kernels_x87.jsonl
fi
if [[ $STAGE == kernels_ab ]]; then
  run timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels_u2.jsonl 2> gpurun_out/bench_kernels.err || exit 1
  MVX_PROG_U1=1 run timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels_u1.jsonl 2>> gpurun_out/bench_kernels.err || exit 1
  run timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels_u2b.jsonl 2>> gpurun_out/bench_kernels.err || exit 1
  MVX_PROG_U1=1 run timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels_u1b.jsonl 2>> gpurun_out/bench_kernels.err || exit 1
  for f in u2 u1 u2b u1b; do echo "-- $f"; cut -c1-200 gpurun_out/bench_kernels_$f.jsonl; done
fi
