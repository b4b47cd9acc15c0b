#!/bin/bash
# b1 GRU-conv tactic sweep (graph-timed, no host launch gaps) + a serialized SF b1 timeline (run under gpurun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 300 python3 tools/conv_bench.py --graph --iters 40 --shapes zr1,q1,fh1,zr8l,q8l,zr32,q32,fhrt \
  --cfgs=-1,0,1,3,4,5,7,8,14,15,16,17 --splits=1,0,2,3,4,6,8,-1 > gpurun_out/tl/r3_sweep.txt 2>&1 || exit 1
export SA_PLAN_CACHE=/tmp/sa_plan_sfser.txt SA_RAFT_PARALLEL=0
timeout -k 10 180 python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 10 > gpurun_out/tl/r3a_sfser_time.log 2>&1 || exit 1
cp /tmp/sa_plan_sfser.txt gpurun_out/tl/r3a_plan_sf.txt
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_sfser -o run -- \
  python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 3 > gpurun_out/tl/r3a_sfser_prof.log 2>&1 || exit 1
cp $(find /tmp/tl_sfser -name "*kernel_trace.csv" | head -1) gpurun_out/tl/r3a_sfser_kernels.csv

timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_cache_gpu.py > gpurun_out/tl/r3_plan_tests.log 2>&1 || exit 1
echo tests-done
