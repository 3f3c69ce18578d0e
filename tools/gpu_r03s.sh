# order-256 tridiagonalisation (512-thread lower-block grid): syev tests, (x+y).round(128) timing with the
# eigensolver at 256 (XRS_SYEV_MAX=256) and its kernel stats
set -o pipefail
D=gpurun_out/r03s
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -q --timeout 100 tests/test_syev_gpu.py > $D/tests.log 2>&1 &&
SUM=1 TARGET=128 REPS=3 XRS_SYEV_MAX=256 XRS_DEBUG_ROUND=1 timeout -k 10 150 python -u tools/trunc_profile.py > $D/sum128_eig.txt 2>&1 &&
SUM=1 TARGET=128 REPS=3 XRS_SYEV_MAX=256 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_sum128 -o run -- python3 tools/trunc_profile.py > $D/prof_sum128.log 2>&1 &&
TARGET=64 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64.txt 2>&1 &&
XRS_SYEV_STAMPS=1 timeout -k 10 120 python -u tools/syev_stamps.py > $D/stamps.txt 2>&1
