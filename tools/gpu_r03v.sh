# fused permuted-operand contraction: its tests, then the cfg1 timing (bench extras only) and a kernel trace
set -o pipefail
D=gpurun_out/r03v
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_api_gpu.py tests/test_reference_ports_gpu.py tests/test_als_gpu.py tests/test_ttoperator_gpu.py > $D/tests.log 2>&1 ;
timeout -k 10 200 python -u tools/cfg1_probe.py > $D/cfg1.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 tools/cfg1_probe.py > $D/prof.log 2>&1
