#!/bin/bash
# 64-deep K-steps (XRS_GLDS_BK=${BKV:-64}) vs 32: GEMM + TT parity, TT-shape GEMM timings, headline step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5"
XRS_GLDS_BK=${BKV:-64} timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_tt_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/bk_tests.log 2>&1 \
  && tail -1 gpurun_out/bk_tests.log \
  && timeout -k 10 120 python tools/gemm_tt_bench.py > gpurun_out/bk32_gemm.log 2>&1 \
  && XRS_GLDS_BK=${BKV:-64} timeout -k 10 120 python tools/gemm_tt_bench.py > gpurun_out/bk64_gemm.log 2>&1 \
  && paste gpurun_out/bk32_gemm.log gpurun_out/bk64_gemm.log | cut -c1-220 \
  && timeout -k 10 120 $B > gpurun_out/bk32.json \
  && XRS_GLDS_BK=${BKV:-64} timeout -k 10 120 $B > gpurun_out/bk64.json \
  && for f in 32 64; do python -c "import json,sys; d=json.load(open('gpurun_out/bk$f.json')); r=d['roofline']; print('$f', d['ms_per_step'], d['config']['sequential_ms_per_step'], r['frac'], r['avg_launch_us'], r['overlapped_step']['frac'])"; done
rc=$?
tail -3 gpurun_out/bk_tests.log
exit $rc
