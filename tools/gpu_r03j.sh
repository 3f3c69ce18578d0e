# Jacobi cross-round phase stamps (svd_sweeps with XRS_SVD_TIMING) + the changed GPU tests
set -o pipefail
D=gpurun_out/r03j
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
XRS_SVD_TIMING=1 timeout -k 10 120 python -u tools/svd_sweeps.py > $D/svd_sweeps.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_factorisations_gpu.py tests/test_ttoperator_gpu.py tests/test_round_general_gpu.py > $D/tests.log 2>&1
