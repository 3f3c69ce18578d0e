#!/bin/bash
# PMC passes over a short bench run (FETCH_SIZE and WRITE_SIZE need separate passes on gfx950), then the
# kernel-trace + stats pass of the same command. Each pass has its own time limit; stop at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
CMD="python3 bench.py --no-cpu --no-cfg5 --steps 3 --warmup 1"
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o p --output-format csv -- $CMD > gpurun_out/pmc/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o p --output-format csv -- $CMD > gpurun_out/pmc/write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/mfma -o p --output-format csv -- $CMD > gpurun_out/pmc/mfma.log 2>&1 && \
echo "pmc ok"
