#!/bin/bash
# A/B of a runtime environment variable that HIP reads at initialisation (so one process per setting), on the
# engine's frame time (tools/run_engine.py), alternating settings; the first run tunes into a shared plan file.
#   VAR=HIP_FORCE_DEV_KERNARG VALUES="unset 1" MODELS="raftstereo-sceneflow hitnet-d400" ROUNDS=2 bash tools/gpu/env_ab.sh tag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-envab}
mkdir -p gpurun_out/$T
for m in ${MODELS:-raftstereo-sceneflow}; do
  export SA_PLAN_CACHE=/tmp/sa_plan_env_$m.txt
  timeout -k 10 200 python3 tools/run_engine.py --model $m --batch ${BATCH:-1} --frames 3 > gpurun_out/$T/tune_$m.log 2>&1 || exit 1
  for r in $(seq ${ROUNDS:-2}); do
    for v in ${VALUES:-unset 1}; do
      if [ "$v" = unset ]; then
        env -u $VAR timeout -k 10 120 python3 tools/run_engine.py --model $m --batch ${BATCH:-1} --frames ${FRAMES:-40} \
          > gpurun_out/$T/run.log 2>&1 || exit 1
      else
        env $VAR=$v timeout -k 10 120 python3 tools/run_engine.py --model $m --batch ${BATCH:-1} --frames ${FRAMES:-40} \
          > gpurun_out/$T/run.log 2>&1 || exit 1
      fi
      echo "$VAR=$v $(grep ms/step gpurun_out/$T/run.log)"
    done
  done
done
