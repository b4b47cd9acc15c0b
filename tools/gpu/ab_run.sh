#!/bin/bash
# Focused GPU check (run under gpurun): selected pytest node ids, then an in-process A/B of one engine knob.
#   TESTS="tests/a.py tests/b.py::x" KNOB=SA_X VALUES=0,1 MODEL=raftstereo-sceneflow BATCH=1 bash tools/gpu/ab_run.sh tag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-ab}
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -v -rfEP --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
  prc=$?
  echo "pytest rc=$prc"; grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -3
  case $prc in 0|1) ;; *) exit $prc ;; esac
fi
if [ -n "$KNOB" ]; then
  timeout -k 10 400 python3 -u tools/ab_engine.py --knob $KNOB --values ${VALUES:-0,1} --model ${MODEL:-raftstereo-sceneflow} \
      --batch ${BATCH:-1} --rounds ${ROUNDS:-6} ${CLEAR:+--clear-plan} > gpurun_out/$T/ab.log 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/$T/ab.log; exit 1; }
  tail -${TAILN:-4} gpurun_out/$T/ab.log
fi
exit ${prc:-0}
