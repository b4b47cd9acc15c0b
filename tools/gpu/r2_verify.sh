set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/diag/tune_verify.py raftstereo-sceneflow:1 raftstereo-realtime:1 crestereo-iter10:1 hitnet-d400:1 hitnet-xl:1 fastacvnet-plus:1 raftstereo-sceneflow:8 --reps 2 > gpurun_out/tune_verify.log 2>&1; rc=$?
grep -v "^\[I\]" gpurun_out/tune_verify.log | tail -40
exit $rc
