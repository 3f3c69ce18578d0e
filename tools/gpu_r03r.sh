# eigensolver v3 (2-barrier sytrd; latency-hidden stebz/stein, 256 threads): quick check
set -o pipefail
D=gpurun_out/r03r
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -q --timeout 100 tests/test_syev_gpu.py > $D/tests.log 2>&1 &&
XRS_SYEV_STAMPS=1 timeout -k 10 120 python -u tools/syev_stamps.py > $D/stamps.txt 2>&1 &&
TARGET=64 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64.txt 2>&1 &&
TARGET=64 REPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_flat64 -o run -- python3 tools/trunc_profile.py > $D/prof_flat64.log 2>&1
