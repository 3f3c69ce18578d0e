cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06d; mkdir -p $D
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $D/p1 -o p --output-format csv -- python3 tools/dot32_one.py 10 > $D/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $D/p2 -o p --output-format csv -- python3 tools/dot32_one.py 10 > $D/p2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $D/p3 -o p --output-format csv -- python3 tools/dot32_one.py 10 > $D/p3.log 2>&1
