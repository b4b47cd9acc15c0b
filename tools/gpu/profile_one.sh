#!/bin/bash
# One kernel-trace profile (run under gpurun):  NAME=sf_b8s MODEL=raftstereo-sceneflow BATCH=8 FRAMES=3 bash tools/gpu/profile_one.sh
# Extra env (e.g. SA_RAFT_PARALLEL=0 SA_RAFT_PIPELINE=0 for a serialized frame) passes through.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export SA_PLAN_CACHE=/tmp/sa_plan_$NAME.txt
rm -f $SA_PLAN_CACHE
timeout -k 10 120 python3 tools/run_engine.py --model $MODEL --batch $BATCH --frames 1 > gpurun_out/prof_${NAME}_tune.log 2>&1 || exit 1
timeout -k 10 240 python3 tools/run_engine.py --model $MODEL --batch $BATCH --frames 10 > gpurun_out/prof_${NAME}_time.log 2>&1 || exit 1
rm -rf gpurun_out/prof_$NAME
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$NAME -o run -- \
  python3 tools/run_engine.py --model $MODEL --batch $BATCH --frames $FRAMES > gpurun_out/prof_$NAME.log 2>&1 || exit 1
db=$(find gpurun_out/prof_$NAME -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" --frames $(( FRAMES + 3 )) --by-grid --top 45 > gpurun_out/prof_$NAME.txt
rm -rf gpurun_out/prof_$NAME
