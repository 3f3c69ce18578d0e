# k_gemm_glds: GEMM parity tests, then the TT-shape timing per variant and workgroup timelines
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread -k gemm > gpurun_out/glds_t1.log 2>&1
rc=$?; tail -n 5 gpurun_out/glds_t1.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-0,256 -1,256 1,256 3,256 4,256 6,256 7,256}; do
  XRS_GEMM_GLDS=$v timeout -k 10 120 python -u tools/gemm_tt_bench.py > gpurun_out/glds_b$v.log 2>&1 || exit 1
  echo "== glds $v"; cat gpurun_out/glds_b$v.log
done
for v in ${TRACES:--1,256 6,256}; do
  XRS_GEMM_GLDS=$v timeout -k 10 120 python -u tools/gemm_trace.py > gpurun_out/gtr_$v.log 2>&1 || exit 1
  echo "== trace $v"; grep rep2 gpurun_out/gtr_$v.log
done
