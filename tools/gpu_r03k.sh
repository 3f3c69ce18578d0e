# FP32-seeded Jacobi rotations: A/B of sweeps, per-round phases and truncating rounds; SVD/round tests
set -o pipefail
D=gpurun_out/r03k
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
XRS_SVD_TIMING=1 timeout -k 10 120 python -u tools/svd_sweeps.py > $D/svd_fast.txt 2>&1 &&
XRS_SVD_EXACT_ROT=1 XRS_SVD_TIMING=1 timeout -k 10 120 python -u tools/svd_sweeps.py > $D/svd_exact.txt 2>&1 &&
GRADED=0.8 TARGET=64 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/graded64_fast.txt 2>&1 &&
XRS_SVD_EXACT_ROT=1 GRADED=0.8 TARGET=64 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/graded64_exact.txt 2>&1 &&
TARGET=64 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64_fast.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_factorisations_gpu.py tests/test_ttoperator_gpu.py tests/test_round_general_gpu.py tests/test_tt_gpu.py tests/test_indexed_factorisations_gpu.py tests/test_cfg5_gpu.py > $D/tests.log 2>&1
