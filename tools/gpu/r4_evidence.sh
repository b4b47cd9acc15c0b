#!/bin/bash
# Round-4 evidence pass (run under gpurun): host-overhead split of the timed region, then b8 kernel profiles of the
# sceneflow step at HEAD (default schedule and serialized).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
SA_HOST_TIMES=1 timeout -k 10 300 python3 -u tools/host_overhead.py > gpurun_out/ev/host_overhead.jsonl 2> gpurun_out/ev/host_overhead.err || exit 1
NAME=sf_b8 MODEL=raftstereo-sceneflow BATCH=8 FRAMES=3 bash tools/gpu/profile_one.sh || exit 1
NAME=sf_b8_serial MODEL=raftstereo-sceneflow BATCH=8 FRAMES=3 SA_RAFT_PARALLEL=0 SA_RAFT_PIPELINE=0 bash tools/gpu/profile_one.sh || exit 1
cp gpurun_out/prof_sf_b8*.txt gpurun_out/ev/
