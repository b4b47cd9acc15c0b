set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in raftstereo-realtime raftstereo-sceneflow; do timeout -k 10 200 python -u tools/diag/latency_parts.py --model $m --frames 30 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/lat_parts.log
nproc
