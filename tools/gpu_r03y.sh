# final check at HEAD: full GPU suite and smoke
set -o pipefail
D=gpurun_out/r03y
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 480 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $D/tests.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
