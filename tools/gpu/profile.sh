#!/bin/bash
# Kernel-trace profiles of the RAFT-Stereo presets + conv micro-benchmark (run under gpurun).
#   gpurun --timeout 900 -- 'bash tools/gpu/profile.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 || exit 1
prof() {  # name model batch frames
  rm -rf gpurun_out/prof_$1
  # tune once outside the profiler (plan persisted), so the trace holds only steady-state frames
  export SA_PLAN_CACHE=/tmp/sa_plan_$1.txt
  rm -f $SA_PLAN_CACHE
  timeout -k 10 120 python3 tools/run_engine.py --model $2 --batch $3 --frames 1 > /dev/null 2>&1 || return 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$1 -o run -- \
    python3 tools/run_engine.py --model $2 --batch $3 --frames $4 > gpurun_out/prof_$1.log 2>&1 || return 1
  db=$(find gpurun_out/prof_$1 -name "*.db" | head -1)
  python3 tools/prof_summary.py "$db" --frames $(( $4 + 2 )) --by-grid --top 45 > gpurun_out/prof_$1.txt
  rm -rf gpurun_out/prof_$1
}
prof ${P1:-sf_b1} ${M1:-raftstereo-sceneflow} ${B1:-1} 5 && \
prof ${P2:-sf_b8} ${M2:-raftstereo-sceneflow} ${B2:-8} 3 && \
prof ${P3:-rt_b1} ${M3:-raftstereo-realtime} ${B3:-1} 10
