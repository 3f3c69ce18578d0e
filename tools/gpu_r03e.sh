# general round (accurate right singular vectors) + DMRG/ALS tests + Jacobi sweep counts
set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_round_general_gpu.py tests/test_als_gpu.py > gpurun_out/r03e/tests.log 2>&1
GRADED=0.8 TARGET=64 REPS=4 timeout -k 10 120 python -u tools/trunc_profile.py > gpurun_out/r03e/graded64.txt 2>&1 &&
GRADED=0.8 TARGET=0 EPS=1e-8 REPS=4 XRS_DEBUG_ROUND=1 timeout -k 10 120 python -u tools/trunc_profile.py > gpurun_out/r03e/graded_eps.txt 2>&1 &&
timeout -k 10 120 python -u tools/svd_sweeps.py > gpurun_out/r03e/svd_sweeps.txt 2>&1
