# PMC passes (one rocprofv3 --pmc run each) over single TT-shape GEMMs: XRS_GEMM_GLDS variant x shape
set -o pipefail
mkdir -p gpurun_out/pmcg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for cfg in ${PMC_CFGS:-"6,256:NN wide" "-1,256:Gram M^T" "-1,256:right chain"}; do
  v=${cfg%%:*}; shape=${cfg#*:}; tag=$(echo "$v$shape" | tr -c 'a-zA-Z0-9' '_')
  for p in 1 2; do
    eval C=\$P$p
    XRS_GEMM_GLDS=$v XRS_BENCH_ONLY="$shape" timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/pmcg/$tag/p$p -o p --output-format csv -- python3 tools/gemm_tt_bench.py > gpurun_out/pmcg/$tag.p$p.log 2>&1 || exit 1
  done
  echo "== $v $shape"; python3 tools/pmc_gemm.py gpurun_out/pmcg/$tag
done
