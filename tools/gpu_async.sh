#!/bin/bash
# Async inner product + triangular transforms: parity tests, then the headline step overlapped /
# sequential / without triangular skipping, host timings, and a kernel trace of the overlapped step.
# Each GPU step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5"
timeout -k 10 300 python -u -m pytest tests/test_tt_gpu.py tests/test_reference_ports_gpu.py tests/test_cfg5_gpu.py tests/test_api_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/async_tests.log 2>&1 \
  && tail -2 gpurun_out/async_tests.log \
  && timeout -k 10 120 $B > gpurun_out/async_overlap.json \
  && timeout -k 10 120 $B --no-overlap > gpurun_out/async_seq.json \
  && XRS_NO_GEMM_PAIR=1 timeout -k 10 120 $B > gpurun_out/async_nopair.json \
  && XRS_NO_GEMM_PAIR=1 timeout -k 10 120 $B --no-overlap > gpurun_out/async_nopair_seq.json \
  && timeout -k 10 120 python tools/host_timing.py > gpurun_out/host_timing2.log 2>&1 && cat gpurun_out/host_timing2.log \
  && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_async -o bench --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras --steps 10 --warmup 3 > gpurun_out/prof_async.log 2>&1 \
  && for f in overlap seq nopair nopair_seq; do python -c "import json,sys; d=json.load(open('gpurun_out/async_$f.json')); print('$f', d['ms_per_step'], d['config']['sequential_ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"; done
rc=$?
tail -5 gpurun_out/async_tests.log
exit $rc
