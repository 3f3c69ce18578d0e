# tridiagonal eigensolver: 256-thread grid (<= 128), lower-block 1024-thread grid (<= 256); unit tests,
# stamps, flat round(64) A/B against the 1024-thread grid, (x + y).round(128) with and without the solver
set -o pipefail
D=gpurun_out/r03q
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -v --timeout 100 tests/test_syev_gpu.py > $D/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $D/tests.log
[ $rc -le 1 ] || exit $rc
XRS_SYEV_STAMPS=1 timeout -k 10 120 python -u tools/syev_stamps.py > $D/stamps.txt 2>&1 &&
TARGET=64 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64.txt 2>&1 &&

SUM=1 TARGET=128 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/sum128_eig.txt 2>&1 &&
XRS_SYEV_MAX=128 SUM=1 TARGET=128 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/sum128_jacobi.txt 2>&1 &&
SUM=1 TARGET=128 REPS=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_sum128 -o run -- python3 tools/trunc_profile.py > $D/prof_sum128.log 2>&1
