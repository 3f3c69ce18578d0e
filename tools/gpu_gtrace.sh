# glds kernel: normal (tools/trace) vs compute-only (tools/trace2) workgroup timelines, per-step cycles
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in ${LIBS:-trace trace2}; do
  for v in ${TRACES:--1,256 6,256}; do
    XRS_LIB_PATH=$PWD/tools/$lib/libxerus_amd.so XRS_GEMM_GLDS=$v timeout -k 10 120 python -u tools/gemm_trace.py > gpurun_out/gtr2_${lib}_$v.log 2>&1 || exit 1
    echo "== $lib glds $v"; grep -A1 rep2 gpurun_out/gtr2_${lib}_$v.log | grep -B1 cycles | cut -c1-150
  done
done
