#!/bin/bash
# Split-K rule A/B: GEMM/TT parity under the new rule, alternating sequential/overlapped steps, cfg5 once each way.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_tt_gpu.py tests/test_cfg5_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
AB="XRS_GLDS_SPLIT_OLD=1" bash tools/gpu_ab_seq.sh || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 10 --warmup 3 > gpurun_out/c5_new.json || exit 1
XRS_GLDS_SPLIT_OLD=1 timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 10 --warmup 3 > gpurun_out/c5_old.json || exit 1
for f in new old; do python -c "import json; d=json.load(open('gpurun_out/c5_$f.json')); print('$f', d['ms_per_step'], d['cfg5'].get('ms_per_round', d['cfg5']))"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o bench --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras --steps 10 --warmup 3 > gpurun_out/prof_ab.log 2>&1
