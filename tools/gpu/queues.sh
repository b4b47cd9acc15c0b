#!/bin/bash
# Frame time of each preset with the graph executor's queue count forced (DEBUG_HIP_FORCE_GRAPH_QUEUES, read at HIP
# initialisation, so one process per setting; the first run tunes into a shared plan file):
#   MODELS="raftstereo-sceneflow crestereo-iter10" QS="0 1 2" bash tools/gpu/queues.sh tag
# QS value 0 = the runtime default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-queues}
mkdir -p gpurun_out/$T
for m in ${MODELS:-raftstereo-sceneflow raftstereo-realtime crestereo-iter10 hitnet-d400 fastacvnet-plus}; do
  export SA_PLAN_CACHE=/tmp/sa_plan_q_$m.txt
  timeout -k 10 200 python3 tools/run_engine.py --model $m --frames 3 > gpurun_out/$T/tune_$m.log 2>&1 || exit 1
  for q in ${QS:-0 1 0 1}; do
    if [ "$q" = 0 ]; then
      timeout -k 10 120 python3 tools/run_engine.py --model $m --frames ${FRAMES:-40} > gpurun_out/$T/run.log 2>&1 || exit 1
    else
      DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 120 python3 tools/run_engine.py --model $m --frames ${FRAMES:-40} \
        > gpurun_out/$T/run.log 2>&1 || exit 1
    fi
    echo "queues=$q $(grep ms/step gpurun_out/$T/run.log)"
  done
done
