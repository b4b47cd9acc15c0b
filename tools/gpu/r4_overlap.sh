#!/bin/bash
# Data-parallel step overlap at HEAD defaults (run under gpurun): bench.py's DP step at world 1
# with the RCCL all-gather forced on (SA_DP_GATHER_WORLD1=1) against the plain step, then a kernel + memory-copy
# trace of the forced step summarised by tools/overlap_report.py (share of every H2D copy / RCCL kernel that runs
# while a compute kernel runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ov; mkdir -p $O
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-latency > /dev/null 2>&1 || exit 1  # tune once
for r in $([ "${SKIP_AB:-0}" = 1 ] || echo 1 2); do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-latency > $O/plain_$r.log 2>&1 || exit 1
  SA_DP_GATHER_WORLD1=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-latency > $O/gather_$r.log 2>&1 || exit 1
done
for f in $O/plain_1 $O/gather_1 $O/plain_2 $O/gather_2; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f.log)"; done
rm -rf /tmp/ovp
SA_DP_GATHER_WORLD1=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d /tmp/ovp -o run -- python3 bench.py --steps 6 --warmup 2 --no-latency > $O/trace.log 2>&1 || exit 1
echo "== bench.py DP step, world 1, gather forced (HEAD defaults), last 6 steps"
python3 tools/overlap_report.py /tmp/ovp --last-ms 250 --dump $O/window.csv | tee $O/overlap.txt
head -3 /tmp/ovp/*/*kernel_trace.csv > $O/kernel_trace_head.txt 2>/dev/null || head -3 /tmp/ovp/*kernel_trace.csv > $O/kernel_trace_head.txt
