#!/bin/bash
# Round-3 profile set (same passes as pmc_r02.sh): FETCH_SIZE / WRITE_SIZE calibration of 8-B loads/stores (tools/fetch_calib.hip), the
# PMC passes of the step-only bench (FETCH, WRITE, MFMA busy; one pass each), then the kernel-trace +
# stats pass of the same command. Each pass has its own time limit; stop at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc3
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o gpurun_out/pmc3/fetch_calib || exit 1
CMD="python3 bench.py --no-cpu --no-cfg5 --no-extras --steps 3 --warmup 1"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3/calf -o p --output-format csv -- gpurun_out/pmc3/fetch_calib > gpurun_out/pmc3/calf.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc3/calw -o p --output-format csv -- gpurun_out/pmc3/fetch_calib > gpurun_out/pmc3/calw.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3/fetch -o p --output-format csv -- $CMD > gpurun_out/pmc3/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc3/write -o p --output-format csv -- $CMD > gpurun_out/pmc3/write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc3/mfma -o p --output-format csv -- $CMD > gpurun_out/pmc3/mfma.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc3/trace -o bench --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras > gpurun_out/pmc3/trace.log 2>&1 && \
echo "pmc ok"
