# fresh kernel-trace summaries for the other model families at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
run() { NAME=$1 MODEL=$2 BATCH=$3 FRAMES=$4 bash tools/gpu/profile_one.sh || return 1; }
run cre10_b1 crestereo-iter10 1 5 && run hit_b1 hitnet-d400 1 10 && run hitxl_b1 hitnet-xl 1 10 && run facv_b1 fastacvnet-plus 1 10
for f in gpurun_out/prof_cre10_b1.txt gpurun_out/prof_hit_b1.txt gpurun_out/prof_hitxl_b1.txt gpurun_out/prof_facv_b1.txt; do echo "== $f"; head -n 1 $f; done
