set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
NAME=sf_b1_r2c MODEL=raftstereo-sceneflow BATCH=1 FRAMES=5 bash tools/gpu/profile_one.sh && \
SA_RAFT_PARALLEL=0 NAME=sf_b1_r2c_serial MODEL=raftstereo-sceneflow BATCH=1 FRAMES=5 bash tools/gpu/profile_one.sh && \
head -30 gpurun_out/prof_sf_b1_r2c_serial.txt && grep -h "ms/step" gpurun_out/prof_sf_b1_r2c*_time.log
