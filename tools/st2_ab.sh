#!/bin/bash
# A/B of XRS_GLDS_ST2 masks (2 LDS stages, two workgroups per CU; bit 0 products, bit 1 Grams, bit 2 the
# one-workgroup split-K rule) on the bench step (headline + sequential), alternating, 2 rounds.
#   tools/st2_ab.sh TAG MASK [MASK ...]
set -o pipefail
O=gpurun_out/${1:-st2ab}; shift; mkdir -p $O
for k in 1 2; do
  for v in "$@"; do
    XRS_GLDS_ST2=$v timeout -k 10 200 python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5 > $O/bench_st2_${v}_$k.json 2> $O/bench_st2_${v}_$k.err || exit 1
  done
done
