# b1 sceneflow with the frame serialized on one stream: true per-kernel cost at batch 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
SA_RAFT_PARALLEL=0 NAME=sf_b1_serial MODEL=raftstereo-sceneflow BATCH=1 FRAMES=5 bash tools/gpu/profile_one.sh && \
head -45 gpurun_out/prof_sf_b1_serial.txt && grep -h "ms" gpurun_out/prof_sf_b1_serial_time.log | tail -3
