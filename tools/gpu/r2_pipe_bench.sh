# bench.py A/B of the cross-iteration pipeline at b8 (SA_RAFT_PIPELINE 0 vs 2), separate processes interleaved;
# GATHER=1 forces the RCCL all-gather path at world size 1 (the DP step's stream / queue usage)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
G=${GATHER:-0}
for r in 1 2; do for m in 0 2; do
  SA_DP_GATHER_WORLD1=$G SA_RAFT_PIPELINE=$m timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-latency 2>/dev/null | grep '^{' > gpurun_out/pb_one.json || exit 1
  python3 - "$G" "$m" "$r" <<'PY'
import json, sys
d = json.load(open("gpurun_out/pb_one.json"))
print(f"gather {sys.argv[1]} pipeline {sys.argv[2]} round {sys.argv[3]}: {d['value']} FPS {d['ms_per_step']} ms/step allgather_ms {d.get('allgather_ms')}")
PY
done; done | tee gpurun_out/pipe_bench_g$G.log
