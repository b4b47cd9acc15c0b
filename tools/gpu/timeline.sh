#!/bin/bash
# Kernel-trace timelines of batch-1 frames (run under gpurun):  bash tools/gpu/r3_timeline.sh [tag]
# For each model: tune once into a plan file, then a csv kernel trace of a few graph replays, summarised by
# tools/timeline.py (frame span / busy / idle, per-iteration spans, critical chain).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r4}
mkdir -p gpurun_out/tl
run() {  # name model iter-marker [batch]
  local name=$1 model=$2 marker=$3 batch=${4:-1}
  export SA_PLAN_CACHE=/tmp/sa_plan_$name.txt
  timeout -k 10 180 python3 tools/run_engine.py --model $model --batch $batch --frames 20 > gpurun_out/tl/${TAG}_${name}_time.log 2>&1 || return 1
  rm -rf /tmp/tl_$name
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_$name -o run -- \
    python3 tools/run_engine.py --model $model --batch $batch --frames 4 > gpurun_out/tl/${TAG}_${name}_prof.log 2>&1 || return 1
  python3 tools/timeline.py /tmp/tl_$name --iter-marker "$marker" --chain 40 --kernel-stats 40 > gpurun_out/tl/${TAG}_${name}.txt 2>&1 || return 1
  cp $(find /tmp/tl_$name -name "*kernel_trace.csv" | head -1) gpurun_out/tl/${TAG}_${name}_kernels.csv
}
if [ -n "$ONLY" ]; then  # one preset by its short name
  case $ONLY in
    sf) run sf raftstereo-sceneflow motion_encoder ;;
    sf8) run sf8 raftstereo-sceneflow motion_encoder 8 ;;
    rt) run rt raftstereo-realtime motion_encoder ;;
    cre10) run cre10 crestereo-iter10 "" ;;
    hit) run hit hitnet-d400 "" ;;
    facv) run facv fastacvnet-plus "" ;;
    *) echo "ONLY=$ONLY: sf sf8 rt cre10 hit facv"; exit 2 ;;
  esac && echo done
  exit $?
fi
run sf raftstereo-sceneflow motion_encoder && \
run sf8 raftstereo-sceneflow motion_encoder 8 && \
run rt raftstereo-realtime motion_encoder && \
run cre10 crestereo-iter10 "" && \
run hit hitnet-d400 "" && \
run facv fastacvnet-plus "" && \
echo done
