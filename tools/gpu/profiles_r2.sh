# Fresh kernel-trace summaries at HEAD for every model family.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
run() { NAME=$1 MODEL=$2 BATCH=$3 FRAMES=$4 bash tools/gpu/profile_one.sh || return 1; }
run sf_b1 raftstereo-sceneflow 1 5 && \
run rt_b1 raftstereo-realtime 1 10 && \
run sf_b8 raftstereo-sceneflow 8 3 && \
SA_RAFT_PARALLEL=0 run sf_b8_serial raftstereo-sceneflow 8 3 && \
run cre10_b1 crestereo-iter10 1 5 && \
run hit_b1 hitnet-d400 1 10 && \
run hitxl_b1 hitnet-xl 1 10 && \
run facv_b1 fastacvnet-plus 1 10
for f in gpurun_out/prof_*.txt; do echo "== $f"; head -3 $f; done
