#!/bin/bash
# SVD / factorisation parity, then the bench with its extras (cfg3 truncating rounds, API SVD timings).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 python -u -m pytest tests/test_factorisations_gpu.py tests/test_tt_gpu.py tests/test_kernels_gpu.py tests/test_reference_ports_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1 \
  && tail -1 gpurun_out/svd_tests.log \
  && timeout -k 10 300 python bench.py --no-cpu --no-cfg5 > gpurun_out/svd_bench.json \
  && python -c "import json; d=json.load(open('gpurun_out/svd_bench.json')); print(d['ms_per_step'], d['cfg3'], d['svd'])"
rc=$?
tail -3 gpurun_out/svd_tests.log
exit $rc
