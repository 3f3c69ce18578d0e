#!/bin/bash
# A/B of one environment switch: GEMM + TT parity under $TESTENV (default: the default code), then the headline step twice
# each way (default, $AB) alternating, and a kernel trace of the default step.
# Usage: AB="XRS_REDUCE_V1=1" bash tools/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5"
env $TESTENV timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_tt_gpu.py tests/test_cfg5_gpu.py tests/test_reference_ports_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 \
  && tail -1 gpurun_out/ab_tests.log \
  && timeout -k 10 120 $B > gpurun_out/ab_def1.json \
  && env $AB timeout -k 10 120 $B > gpurun_out/ab_alt1.json \
  && timeout -k 10 120 $B > gpurun_out/ab_def2.json \
  && env $AB timeout -k 10 120 $B > gpurun_out/ab_alt2.json \
  && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o bench --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras --steps 10 --warmup 3 > gpurun_out/prof_ab.log 2>&1 \
  && for f in def1 alt1 def2 alt2; do python -c "import json,sys; d=json.load(open('gpurun_out/ab_$f.json')); r=d['roofline']; print('$f', d['ms_per_step'], d['config']['sequential_ms_per_step'], r['frac'], r['avg_launch_us'], r['overlapped_step']['frac'])"; done
rc=$?
tail -3 gpurun_out/ab_tests.log
exit $rc
