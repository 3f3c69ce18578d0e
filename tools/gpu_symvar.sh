#!/bin/bash
# Symmetric Gram tile variant A/B (XRS_GLDS_SYM_VAR): parity of the TT tests, then the headline step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python bench.py --no-cpu --no-cfg5 --no-extras --steps 30 --warmup 5"
XRS_GLDS_SYM_VAR=5 timeout -k 10 300 python -u -m pytest tests/test_tt_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/symvar_tests.log 2>&1 \
  && tail -1 gpurun_out/symvar_tests.log \
  && timeout -k 10 120 $B > gpurun_out/symvar_def.json \
  && XRS_GLDS_SYM_VAR=5 timeout -k 10 120 $B > gpurun_out/symvar_5.json \
  && timeout -k 10 120 $B > gpurun_out/symvar_def2.json \
  && XRS_GLDS_SYM_VAR=5 timeout -k 10 120 $B > gpurun_out/symvar_52.json \
  && XRS_GLDS_SYM_VAR=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sym5 -o bench --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras --steps 10 --warmup 3 > gpurun_out/prof_sym5.log 2>&1 \
  && for f in def 5 def2 52; do python -c "import json,sys; d=json.load(open('gpurun_out/symvar_$f.json')); r=d['roofline']; print('$f', d['ms_per_step'], d['config']['sequential_ms_per_step'], r['frac'], r['avg_launch_us'], r['overlapped_step']['frac'])"; done
