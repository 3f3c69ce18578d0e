#!/bin/bash
# One GPU session: the -m gpu parity suite, smoke, the bench line and a rocprofv3 kernel-trace
# summary of the bench. Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 \
  && tail -3 gpurun_out/tests_$TAG.log \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  && timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  && cat gpurun_out/bench_$TAG.json \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o bench --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_$TAG.log 2>&1 \
  && echo "profile ok"
rc=$?
tail -25 gpurun_out/tests_$TAG.log 2>/dev/null
exit $rc
