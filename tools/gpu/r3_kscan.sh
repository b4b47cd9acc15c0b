#!/bin/bash
# Fixed vs per-k-step cost of the small-M GRU convs: K scan at M = 1200 / 4800 (graph-timed, and a kernel trace of
# the same run so kernel durations can be separated from dispatch gaps).  Run under gpurun.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
S=1x30x40x64x256k3,1x30x40x128x256k3,1x30x40x256x256k3,1x30x40x512x256k3,1x60x80x64x256k3,1x60x80x256x256k3,1x60x80x512x256k3,1x30x40x256x256k1
timeout -k 10 200 python3 tools/conv_bench.py --graph --iters 20 --shapes $S --cfgs=16,5,3,1 --splits=1,2,4 > gpurun_out/tl/r3_kscan.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/ks -o run -- python3 tools/conv_bench.py --graph --iters 20 --shapes $S --cfgs=16,3 --splits=1,4 > gpurun_out/tl/r3_kscan_prof.log 2>&1 || exit 1
cp $(find /tmp/ks -name "*kernel_stats.csv" | head -1) gpurun_out/tl/r3_kscan_stats.csv
cp $(find /tmp/ks -name "*kernel_trace.csv" | head -1) gpurun_out/tl/r3_kscan_trace.csv

export SA_PLAN_CACHE=/tmp/sa_plan_sf3.txt
SA_RAFT_PIPELINE=3 timeout -k 10 180 python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 20 > gpurun_out/tl/r3b_sf3_time.log 2>&1 || exit 1
timeout -k 10 180 python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 20 > gpurun_out/tl/r3b_sf2_time.log 2>&1 || exit 1
SA_RAFT_PIPELINE=3 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_sf3 -o run -- \
  python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 3 > gpurun_out/tl/r3b_sf3_prof.log 2>&1 || exit 1
cp $(find /tmp/tl_sf3 -name "*kernel_trace.csv" | head -1) gpurun_out/tl/r3b_sf3_kernels.csv
unset SA_PLAN_CACHE
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_raft_modes_gpu.py > gpurun_out/tl/r3b_modes.log 2>&1 || exit 1
echo all-done
