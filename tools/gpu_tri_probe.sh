#!/bin/bash
# Transform GEMMs with / without the triangular K-range skip: kernel traces of the round loop.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tri -o tri -- python3 tools/host_timing.py > gpurun_out/prof_tri.log 2>&1 \
  && XRS_NO_TRI=1 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_notri -o notri -- python3 tools/host_timing.py > gpurun_out/prof_notri.log 2>&1 \
  && echo tri-probe ok
