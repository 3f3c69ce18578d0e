#!/bin/bash
# A/B of XRS_GLDS_XCD_SPLIT (whole split-K slices per XCD) on the bench step, alternating, 2 rounds; then the
# FETCH_SIZE pass of the step with the new mapping.
set -o pipefail
O=gpurun_out/${1:-xcdab}; mkdir -p $O
for k in 1 2; do
  for v in 1 0; do
    XRS_GLDS_XCD_SPLIT=$v timeout -k 10 200 python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5 > $O/bench_x${v}_$k.json 2> $O/bench_x${v}_$k.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc/fetch" -o p --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras --no-overlap --steps 20 --warmup 3 > "$O/pmc_fetch.log" 2>&1
