#!/bin/bash
# GEMM tile-variant sweep under rocprofv3 kernel tracing (one trace per XRS_GEMM_CFG).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for c in "$@"; do
  XRS_GEMM_CFG=$c timeout -k 5 200 rocprofv3 --kernel-trace -d gpurun_out/gsw/$c -o t --output-format csv -- python3 tools/gemm_shapes.py > gpurun_out/gsw_$c.log 2>&1 || exit 1
done
