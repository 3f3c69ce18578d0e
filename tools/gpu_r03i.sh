# full GPU suite + smoke + bench + rocprof of the bench + truncating-round timings (per-edge Jacobi sweeps)
set -o pipefail
D=gpurun_out/r03i
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 &&
GRADED=0.8 TARGET=64 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/graded64.txt 2>&1 &&
GRADED=0.8 TARGET=0 EPS=1e-8 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/graded_eps.txt 2>&1 &&
TARGET=64 REPS=3 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64.txt 2>&1 &&
XRS_SVD_TIMING=1 timeout -k 10 120 python -u tools/svd_sweeps.py > $D/svd_sweeps.txt 2>&1 &&
timeout -k 10 240 python -u bench.py > $D/bench.json 2> $D/bench.err &&
GRADED=0.8 TARGET=64 REPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_g64 -o run -- python3 tools/trunc_profile.py > $D/prof_g64.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_bench -o run -- python3 bench.py > $D/prof_bench.log 2>&1
