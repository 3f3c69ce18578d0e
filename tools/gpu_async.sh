#!/bin/bash
# Async inner product: parity tests, then the headline step with the gated product (default), started at
# once (XRS_DOT_GATE=0) and sequential, and a kernel trace of the default step.
# Each GPU step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5"
timeout -k 10 300 python -u -m pytest tests/test_tt_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/async_tests.log 2>&1 \
  && tail -2 gpurun_out/async_tests.log \
  && timeout -k 10 120 $B > gpurun_out/async_gate.json \
  && XRS_DOT_GATE=0 timeout -k 10 120 $B > gpurun_out/async_nogate.json \
  && timeout -k 10 120 $B > gpurun_out/async_gate2.json \
  && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gate -o bench --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras --steps 10 --warmup 3 > gpurun_out/prof_gate.log 2>&1 \
  && for f in gate nogate gate2; do python -c "import json,sys; d=json.load(open('gpurun_out/async_$f.json')); r=d['roofline']; print('$f', d['ms_per_step'], d['config']['sequential_ms_per_step'], r['frac'], r['avg_launch_us'], r['overlapped_step']['frac'])"; done
rc=$?
tail -3 gpurun_out/async_tests.log
exit $rc
