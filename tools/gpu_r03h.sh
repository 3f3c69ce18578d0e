# full GPU suite + smoke + default bench (JSON line) + rocprof kernel stats of the bench command
set -o pipefail
mkdir -p gpurun_out/r03h
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03h/tests.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03h/smoke.log 2>&1 &&
timeout -k 10 240 python -u bench.py > gpurun_out/r03h/bench.json 2> gpurun_out/r03h/bench.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03h/prof_bench -o run -- python3 bench.py > gpurun_out/r03h/prof_bench.log 2>&1
