#!/bin/bash
# A/B of XRS_GLDS_ST2 (2 LDS stages, two workgroups per CU) against the default 3-stage glds tiles:
# TT-shaped GEMMs back to back, then the bench step (headline + sequential), alternating, 2 rounds.
set -o pipefail
O=gpurun_out/${1:-st2ab}; mkdir -p $O
for k in 1 2; do
  for v in 0 1; do
    XRS_GLDS_ST2=$v timeout -k 10 120 python tools/gemm_tt_bench.py > $O/gemm_st2_${v}_$k.txt 2>&1 || exit 1
    XRS_GLDS_ST2=$v timeout -k 10 200 python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5 > $O/bench_st2_${v}_$k.json 2> $O/bench_st2_${v}_$k.err || exit 1
  done
done
