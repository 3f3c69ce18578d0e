# GEMM workgroup timelines (tools/gemm_trace.py) for forced glds variants (TRACES="v,target ...")
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${TRACES:--1,256 6,256}; do
  XRS_GEMM_GLDS=$v timeout -k 10 120 python -u tools/gemm_trace.py > gpurun_out/gtr_$v.log 2>&1 || exit 1
  echo "== glds $v"; grep -A1 rep2 gpurun_out/gtr_$v.log
done
