# round-3 records: full GPU suite, smoke, default bench line, rocprof kernel stats of it, PMC traffic passes
set -o pipefail
D=${D:-gpurun_out/r03p}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 480 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 &&
timeout -k 10 240 python -u bench.py > $D/bench.json 2> $D/bench.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_bench -o run -- python3 bench.py --no-cpu > $D/prof_bench.log 2>&1 &&
bash tools/pmc_r03.sh > $D/pmc.log 2>&1
