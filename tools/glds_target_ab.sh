#!/bin/bash
# A/B of the glds split-K workgroup target (XRS_GEMM_GLDS="-1,target") on the bench step, alternating, 2 rounds.
#   tools/glds_target_ab.sh TAG TARGET [TARGET ...]
set -o pipefail
O=gpurun_out/${1:-tgtab}; shift; mkdir -p $O
for k in 1 2; do
  for t in "$@"; do
    XRS_GEMM_GLDS="-1,$t" timeout -k 10 200 python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5 > $O/bench_t${t}_$k.json 2> $O/bench_t${t}_$k.err || exit 1
  done
done
