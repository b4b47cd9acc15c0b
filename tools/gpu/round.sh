#!/bin/bash
# Round check under gpurun: the whole GPU test suite (not stopped by the bench), the default bench.py line exactly
# as the round-end driver runs it, then the regression gate against the previous round's driver BENCH_r*.json
# (tools/bench_regress.py, > 3 % worse on any preset fails).  All three statuses are reported; the script fails if
# any failed.  A GPU fault / abort / time limit in pytest ends the call before the bench.
#   gpurun --timeout 1100 -- 'bash tools/gpu/round.sh r5c'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-round}
mkdir -p gpurun_out/$T
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu"}
timeout -k 10 1000 python3 -u -m pytest $PYTEST_ARGS -v -rfEP --durations=25 --timeout 300 --timeout-method thread \
    > gpurun_out/$T/pytest.log 2>&1
prc=$?
echo "pytest rc=$prc"; tail -40 gpurun_out/$T/pytest.log | grep -E "passed|failed|FAILED|ERROR" || true
case $prc in
  0|1) ;;  # 1 = some tests failed: still bench
  *) echo "pytest ended abnormally (rc=$prc): no bench"; exit $prc ;;
esac
[ "${NO_BENCH:-0}" = 1 ] && exit $prc
mkdir -p gpurun_out/$T/plans  # the tuned plans of the b8 step and the 8 batch-1 presets (committed as evidence)
SA_PLAN_DIR=$PWD/gpurun_out/$T/plans timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/bench.log 2>&1
brc=$?
echo "bench rc=$brc"; tail -1 gpurun_out/$T/bench.log | cut -c1-600
grc=0
if [ $brc -eq 0 ]; then
  python3 tools/bench_regress.py gpurun_out/$T/bench.log > gpurun_out/$T/regress.txt 2>&1
  grc=$?
  cat gpurun_out/$T/regress.txt
fi
[ $prc -eq 0 ] && [ $brc -eq 0 ] && [ $grc -eq 0 ]
