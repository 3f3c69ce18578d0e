#!/bin/bash
# Quick GPU iteration: one pytest file (all failures reported) then smoke. Each GPU step time-limited.
set -o pipefail
TAG=${1:-q}
FILE=${2:-tests}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -m pytest $FILE -q -m gpu -rf > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -40 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc2=$?
cat gpurun_out/smoke_$TAG.log | tail -20
exit $(( rc > rc2 ? rc : rc2 ))
