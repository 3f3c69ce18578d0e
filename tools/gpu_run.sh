#!/bin/bash
# One parameterised GPU session (replaces the per-experiment gpu_r03*.sh scripts).
#
#   tools/gpu_run.sh TAG STEP [STEP ...]        outputs under gpurun_out/TAG/
#
# Steps (each under its own time limit; the chain stops at the first failure, nothing runs after it):
#   tests             the whole -m gpu suite                      -> tests.log
#   test:PATH         one test file / node id (-m gpu)            -> test_<n>.log
#   smoke             __graft_entry__.smoke()                     -> smoke.log
#   bench             python bench.py (default line)             -> bench.json
#   benchq            bench.py --no-cpu (no CPU leg)              -> benchq.json
#   trace             rocprofv3 --kernel-trace --stats of the step-only SEQUENTIAL bench
#                     (bench.py --no-cpu --no-cfg5 --no-extras --no-overlap: the roofline pass's step)
#                                                                 -> trace/   (+ roofline.txt)
#   traceov           the same for the headline (overlapped) step -> traceov/
#   tracefull         rocprofv3 of the whole default bench (--no-cpu) -> tracefull/
#   pmc               FETCH_SIZE / WRITE_SIZE calibration + PMC passes over the step-only bench -> pmc/
#   py:SCRIPT[,ARG..] python -u SCRIPT ARG..                       -> py_<n>.txt
#   prof:SCRIPT[,ARG..] rocprofv3 --kernel-trace --stats of python3 SCRIPT ARG.. -> prof_<n>/
# Environment switches for a step go on the gpurun command line (VAR=value tools/gpu_run.sh ...).
set -o pipefail
TAG=${1:?tag}
shift
D=gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$D"
STEPCMD="python3 bench.py --no-cpu --no-cfg5 --no-extras --no-overlap --steps 20 --warmup 3"
n=0
for step in "$@"; do
  n=$((n + 1))
  echo "[gpu_run] step $n: $step" >&2
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > "$D/tests.log" 2>&1
      rc=$?; tail -3 "$D/tests.log" ;;
    test:*)
      timeout -k 10 600 python -u -m pytest "${step#test:}" -v -m gpu -x --timeout 300 --timeout-method thread -rf > "$D/test_$n.log" 2>&1
      rc=$?; tail -15 "$D/test_$n.log" ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$D/smoke.log" 2>&1
      rc=$?; tail -2 "$D/smoke.log" ;;
    bench)
      timeout -k 10 400 python bench.py > "$D/bench.json" 2> "$D/bench.err"
      rc=$?; cut -c1-600 "$D/bench.json" ;;
    benchq)
      timeout -k 10 300 python bench.py --no-cpu > "$D/benchq.json" 2> "$D/benchq.err"
      rc=$?; cut -c1-600 "$D/benchq.json" ;;
    trace)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$D/trace" -o step --output-format csv -- $STEPCMD > "$D/trace.json" 2> "$D/trace.err" \
        && python3 tools/roofline_from_trace.py "$D/trace" "$D/trace.json" > "$D/roofline.txt"
      rc=$?; cat "$D/roofline.txt" 2>/dev/null | tail -12 ;;
    traceov)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$D/traceov" -o step --output-format csv -- python3 bench.py --no-cpu --no-cfg5 --no-extras --steps 20 --warmup 3 > "$D/traceov.json" 2> "$D/traceov.err"
      rc=$? ;;
    tracefull)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$D/tracefull" -o bench --output-format csv -- python3 bench.py --no-cpu > "$D/tracefull.json" 2> "$D/tracefull.err"
      rc=$? ;;
    pmc)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o "$D/fetch_calib" \
      && timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$D/pmc/calf" -o p --output-format csv -- "$D/fetch_calib" > "$D/pmc_calf.log" 2>&1 \
      && timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$D/pmc/calw" -o p --output-format csv -- "$D/fetch_calib" > "$D/pmc_calw.log" 2>&1 \
      && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$D/pmc/fetch" -o p --output-format csv -- $STEPCMD > "$D/pmc_fetch.log" 2>&1 \
      && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$D/pmc/write" -o p --output-format csv -- $STEPCMD > "$D/pmc_write.log" 2>&1 \
      && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$D/pmc/mfma" -o p --output-format csv -- $STEPCMD > "$D/pmc_mfma.log" 2>&1
      rc=$? ;;
    py:*)
      IFS=, read -r -a a <<< "${step#py:}"
      timeout -k 10 300 python -u "${a[@]}" > "$D/py_$n.txt" 2>&1
      rc=$?; tail -20 "$D/py_$n.txt" ;;
    prof:*)
      IFS=, read -r -a a <<< "${step#prof:}"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/prof_$n" -o run --output-format csv -- python3 "${a[@]}" > "$D/prof_$n.txt" 2>&1
      rc=$?; tail -20 "$D/prof_$n.txt" ;;
    *)
      echo "[gpu_run] unknown step $step" >&2; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "[gpu_run] step $n ($step) failed with status $rc; stopping" >&2
    exit $rc
  fi
done
echo "[gpu_run] all steps ok" >&2
