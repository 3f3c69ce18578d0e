set -o pipefail
mkdir -p gpurun_out/r03c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_indexed_factorisations_gpu.py > gpurun_out/r03c/tests.log 2>&1
GRADED=0.8 TARGET=64 REPS=4 timeout -k 10 120 python -u tools/trunc_profile.py > gpurun_out/r03c/graded64.txt 2>&1 &&
GRADED=0.8 TARGET=0 EPS=1e-8 REPS=4 timeout -k 10 120 python -u tools/trunc_profile.py > gpurun_out/r03c/graded_eps.txt 2>&1 &&
TARGET=64 REPS=4 timeout -k 10 120 python -u tools/trunc_profile.py > gpurun_out/r03c/flat64.txt 2>&1 &&
GRADED=0.8 TARGET=64 REPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03c/prof_g64 -o run -- python3 tools/trunc_profile.py > gpurun_out/r03c/prof_g64.log 2>&1
