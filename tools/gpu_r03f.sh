# general round (chain left sweep) tests + dist tests + timings + rocprof split
set -o pipefail
mkdir -p gpurun_out/r03f
export XRS_DEBUG_ROUND=1
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_round_general_gpu.py tests/test_dist_gpu.py tests/test_tt_gpu.py > gpurun_out/r03f/tests.log 2>&1
GRADED=0.8 TARGET=64 REPS=4 timeout -k 10 120 python -u tools/trunc_profile.py > gpurun_out/r03f/graded64.txt 2>&1 &&
GRADED=0.8 TARGET=0 EPS=1e-8 REPS=4 timeout -k 10 120 python -u tools/trunc_profile.py > gpurun_out/r03f/graded_eps.txt 2>&1 &&
unset XRS_DEBUG_ROUND &&
GRADED=0.8 TARGET=64 REPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f/prof_g64 -o run -- python3 tools/trunc_profile.py > gpurun_out/r03f/prof_g64.log 2>&1
