#!/bin/bash
# PMC passes (one counter group per run, rocprofv3 --pmc) + a kernel trace over tools/sgemm_one.py.
#   tools/sgemm_pmc.sh TAG M N K TA TB      outputs under gpurun_out/TAG/
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$D"
CMD="python3 tools/sgemm_one.py $* 100"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$D/trace" -o t --output-format csv -- $CMD > "$D/trace.log" 2>&1 \
&& timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$D/p1" -o p --output-format csv -- $CMD > "$D/p1.log" 2>&1 \
&& timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES -d "$D/p2" -o p --output-format csv -- $CMD > "$D/p2.log" 2>&1
rc=$?
python3 tools/pmc_gemm.py "$D" > "$D/pmc.txt" 2>&1
cat "$D/pmc.txt"
grep -h "k_sgemm" "$D"/trace/*kernel_stats.csv | cut -c1-300
exit $rc
