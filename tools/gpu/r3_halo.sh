#!/bin/bash
# halo-reuse conv tiles: op tests, graph-timed micro-benchmark on the GRU / flow-head shapes, engines (run under gpurun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
T=${1:-r3d}
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "halo or flow_head_tail" > gpurun_out/tl/${T}_halo_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/conv_bench.py --graph --iters 20 --shapes zr1,q1,fh1,zr8l,q8l,zr32,zr8,q8,fh8,zr8s \
  --cfgs=-1,4,5,7,15,16,26,27 --splits=1 > gpurun_out/tl/${T}_halo_bench.txt 2>&1 || exit 1
for model in raftstereo-sceneflow raftstereo-realtime crestereo-iter10; do
  SA_PLAN_CACHE=/tmp/sa_plan_$model.txt timeout -k 10 240 python3 tools/run_engine.py --model $model --batch 1 --frames 2 > /dev/null 2>&1 || exit 1
  SA_PLAN_CACHE=/tmp/sa_plan_$model.txt timeout -k 10 120 python3 tools/run_engine.py --model $model --batch 1 --frames 40 > gpurun_out/tl/${T}_${model}.log 2>&1 || exit 1
  cp /tmp/sa_plan_$model.txt gpurun_out/tl/${T}_plan_${model}.txt
done
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-latency > gpurun_out/tl/${T}_bench_b8.log 2>&1 || exit 1
grep -h "ms/step" gpurun_out/tl/${T}_*.log; tail -1 gpurun_out/tl/${T}_bench_b8.log
