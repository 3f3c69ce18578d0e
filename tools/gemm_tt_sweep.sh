#!/bin/bash
# TT-shape GEMM tile sweep (tools/gemm_tt_bench.py per XRS_GEMM_CFG variant); each run time-limited,
# the chain stops at the first failure. Usage: tools/gemm_tt_sweep.sh TAG cfg1 cfg2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/gemm_tt_bench.py > gpurun_out/gtt_${TAG}_default.log 2>&1 || exit 1
for c in "$@"; do
  XRS_GEMM_CFG=$c timeout -k 10 120 python -u tools/gemm_tt_bench.py > gpurun_out/gtt_${TAG}_$c.log 2>&1 || exit 1
done
cat gpurun_out/gtt_${TAG}_*.log
