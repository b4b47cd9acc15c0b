#!/bin/bash
# Round check under gpurun: the whole GPU test suite first (not stopped by the bench), then the default bench.py line
# exactly as the round-end driver runs it.  Both exit statuses are reported; the script fails if either failed.
# A GPU fault / abort / time limit in pytest ends the call before the bench (no further GPU step after such a status).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r4}
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
[ $prc -eq 0 ] && [ $brc -eq 0 ]
