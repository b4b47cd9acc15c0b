#!/bin/bash
# Multi-rank rehearsal of bench.py on the one-GPU box (run under gpurun): world 2 over gloo with both ranks on the
# same device (RCCL needs distinct GPUs), b8 per rank, latency block off.  Exercises the launcher contract, rank 0's
# plan broadcast (plans_identical_across_ranks), the async all-gather path and the max-over-ranks timing.
#   gpurun --timeout 700 -- 'bash tools/gpu/dp_rehearsal.sh tag'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-dp}
mkdir -p gpurun_out/$T
SA_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-latency \
  > gpurun_out/$T/dp2.log 2>&1
rc=$?
echo "dp rehearsal rc=$rc"
grep '"metric"' gpurun_out/$T/dp2.log | tail -1 | cut -c1-400
exit $rc
