# ADF + measurement operators on the GPU
set -o pipefail
D=gpurun_out/r03l
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_adf_gpu.py tests/test_measurements_cpu.py > $D/tests.log 2>&1
