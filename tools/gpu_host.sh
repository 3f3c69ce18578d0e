#!/bin/bash
# Host-side cost of the step: call timings, launch overhead, round phase marks, and a HIP API trace.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 python tools/host_timing.py > gpurun_out/host_timing.log 2>&1 \
  && cat gpurun_out/host_timing.log \
  && timeout -k 10 120 python tools/launch_overhead.py > gpurun_out/launch_overhead.log 2>&1 \
  && cat gpurun_out/launch_overhead.log \
  && XRS_ROUND_TIMING=1 timeout -k 10 120 python tools/host_timing.py > gpurun_out/host_marks.log 2>&1 \
  && timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/prof_host -o ht -- python3 tools/host_timing.py > gpurun_out/prof_host.log 2>&1 \
  && echo traced
