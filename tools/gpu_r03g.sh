# full GPU suite + smoke + default bench (JSON line) + rocprof kernel stats of the bench command
set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03g/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03g/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r03g/bench.json 2> gpurun_out/r03g/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03g/prof_bench -o run -- python3 bench.py > gpurun_out/r03g/prof_bench.log 2>&1
