# tridiagonal eigensolver for the certified truncation: unit tests, round parity tests, timings (eig vs Jacobi)
set -o pipefail
D=gpurun_out/r03m
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_syev_gpu.py > $D/tests_syev.log 2>&1
rc=$?; echo "rc=$rc" >> $D/tests_syev.log
[ $rc -le 1 ] || exit $rc
TARGET=64 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64_eig.txt 2>&1 &&
XRS_TRUNC_JACOBI=1 TARGET=64 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64_jacobi.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_tt_gpu.py tests/test_round_general_gpu.py tests/test_cfg5_gpu.py tests/test_dist_gpu.py > $D/tests_round.log 2>&1 &&
TARGET=64 REPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_flat64 -o run -- python3 tools/trunc_profile.py > $D/prof_flat64.log 2>&1
