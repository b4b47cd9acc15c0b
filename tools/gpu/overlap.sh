# DP overlap evidence on one GPU: bench.py's multi-GPU step (H2D prefetch on a copy
# stream, async RCCL all-gather, frame graph) at world 1 with the collective forced on, traced with
# kernel + memory-copy tracing; then the 3-stream vs 2-stream engine A/B at batch 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
# warm the plan cache so the trace holds steady-state steps
SA_DP_GATHER_WORLD1=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-latency > /dev/null 2>&1 || exit 1
for pipe in 1 0; do
  rm -rf gpurun_out/ov_$pipe
  SA_RAFT_PIPELINE=$pipe SA_DP_GATHER_WORLD1=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace \
    --output-format csv -d gpurun_out/ov_$pipe -o run -- python3 bench.py --steps 6 --warmup 2 --no-latency \
    > gpurun_out/ov_$pipe.log 2>&1 || exit 1
  echo "== SA_RAFT_PIPELINE=$pipe ($( [ $pipe = 1 ] && echo 3 || echo 2 ) engine streams)"
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov_$pipe.log
  python3 tools/overlap_report.py gpurun_out/ov_$pipe --last-ms 380 | tee gpurun_out/ov_$pipe.txt
  rm -rf gpurun_out/ov_$pipe
done
timeout -k 10 300 python3 tools/ab_engine.py --knob SA_RAFT_PIPELINE --values 1,0 --batch 8 --rounds 4 --frames 4
