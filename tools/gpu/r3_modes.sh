#!/bin/bash
# RAFT b1 schedule / GRU-split A/B + timelines + schedule-equality and GRU-split op tests (run under gpurun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
T=${1:-r3c}
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "gru" > gpurun_out/tl/${T}_optests.log 2>&1 || exit 1
for model in raftstereo-sceneflow raftstereo-realtime; do
  for sp in 0 1; do
    export SA_PLAN_CACHE=/tmp/sa_plan_${model}_$sp.txt SA_RAFT_GRU_SPLIT=$sp
    timeout -k 10 180 python3 tools/run_engine.py --model $model --batch 1 --frames 2 > /dev/null 2>&1 || exit 1
    for m in 2 3 4; do
      SA_RAFT_PIPELINE=$m timeout -k 10 120 python3 tools/run_engine.py --model $model --batch 1 --frames 40 > gpurun_out/tl/${T}_${model}_m${m}_s${sp}.log 2>&1 || exit 1
    done
  done
done
export SA_PLAN_CACHE=/tmp/sa_plan_raftstereo-sceneflow_1.txt SA_RAFT_GRU_SPLIT=1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 SA_RAFT_PIPELINE=4 timeout -k 10 120 python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 40 > gpurun_out/tl/${T}_sf_m4_s1_pc0.log 2>&1 || exit 1
for mm in "raftstereo-sceneflow 4" "raftstereo-realtime 3"; do
  set -- $mm
  export SA_PLAN_CACHE=/tmp/sa_plan_${1}_1.txt
  SA_RAFT_PIPELINE=$2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_$1 -o run -- \
    python3 tools/run_engine.py --model $1 --batch 1 --frames 3 > gpurun_out/tl/${T}_$1_prof.log 2>&1 || exit 1
  cp $(find /tmp/tl_$1 -name "*kernel_trace.csv" | head -1) gpurun_out/tl/${T}_$1_kernels.csv
done
unset SA_PLAN_CACHE SA_RAFT_GRU_SPLIT
for sp in 0 1; do
  SA_PLAN_CACHE=/tmp/sa_plan_cre_$sp.txt SA_CRE_GRU_SPLIT=$sp timeout -k 10 180 python3 tools/run_engine.py --model crestereo-iter10 --batch 1 --frames 2 > /dev/null 2>&1 || exit 1
  SA_PLAN_CACHE=/tmp/sa_plan_cre_$sp.txt SA_CRE_GRU_SPLIT=$sp timeout -k 10 120 python3 tools/run_engine.py --model crestereo-iter10 --batch 1 --frames 40 > gpurun_out/tl/${T}_cre10_s${sp}.log 2>&1 || exit 1
done
timeout -k 10 120 python3 tools/launch_floor.py > gpurun_out/tl/${T}_launch_floor.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_raft_modes_gpu.py > gpurun_out/tl/${T}_modes.log 2>&1 || exit 1
grep -H "ms/step" gpurun_out/tl/${T}_*.log
