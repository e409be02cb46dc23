#!/bin/bash
# Host-operand op pipeline: chunk size sweep (MVX_HOST_CHUNK_MIB; 0 = adaptive)
set -o pipefail
for c in 0 4 8 32 64; do
  MVX_HOST_CHUNK_MIB=$c timeout -k 10 200 python tools/bench_host.py --cases op_pageable,op_pinned --min-mib 32 > gpurun_out/hs_$c.jsonl 2>gpurun_out/hs.err || exit 1
  echo "chunk $c"; cut -c1-120 gpurun_out/hs_$c.jsonl
done
