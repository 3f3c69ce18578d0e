#!/bin/bash
# Sequential-step A/B of one environment switch ($AB), alternating 3 times on the same box.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python bench.py --no-cpu --no-cfg5 --no-extras --steps 50 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 120 $B --no-overlap > gpurun_out/abs_def$i.json || exit 1
  env $AB timeout -k 10 120 $B --no-overlap > gpurun_out/abs_alt$i.json || exit 1
  timeout -k 10 120 $B > gpurun_out/abo_def$i.json || exit 1
  env $AB timeout -k 10 120 $B > gpurun_out/abo_alt$i.json || exit 1
done
for f in abs_def abs_alt abo_def abo_alt; do
  python -c "import json; print('$f', ' '.join('%.4f' % json.load(open('gpurun_out/$f%d.json' % i))['ms_per_step'] for i in (1, 2, 3)))"
done
