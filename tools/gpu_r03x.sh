# v_rcp_f64 accuracy, then the eigensolver with one Newton step in its chains (XRS_SYEV_RCP1=1) vs two
set -o pipefail
D=gpurun_out/r03x
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/rcp_probe > $D/rcp.txt 2>&1 &&
XRS_SYEV_RCP1=1 timeout -k 10 200 python -u -m pytest -q --timeout 100 tests/test_syev_gpu.py > $D/tests_rcp1.log 2>&1 ;
TARGET=64 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64_rcp2.txt 2>&1 &&
XRS_SYEV_RCP1=1 TARGET=64 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64_rcp1.txt 2>&1 &&
TARGET=64 REPS=3 timeout -k 10 120 python -u tools/trunc_profile.py > $D/flat64_rcp2b.txt 2>&1
