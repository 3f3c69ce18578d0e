#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc1 -o p --output-format csv -- python3 tools/gemm_one.py $* > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc2 -o p --output-format csv -- python3 tools/gemm_one.py $* > gpurun_out/pmc2.log 2>&1
