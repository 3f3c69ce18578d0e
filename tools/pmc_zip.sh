#!/bin/bash
# PMC passes over the fused fp32 zipper (tools/dot32_one.py), one counter group per run (gpurun_out/$1/p*)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-zpmc}; mkdir -p $D
run() { timeout -s KILL 90 rocprofv3 --pmc "$@" -d $D/p$N -o p --output-format csv -- python3 tools/dot32_one.py 6 > $D/p$N.log 2>&1; }
N=1; run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD || exit 1
N=2; run TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum || exit 1
N=3; run TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum || exit 1
N=4; run TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum || exit 1
