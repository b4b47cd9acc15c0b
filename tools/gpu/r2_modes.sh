set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 240 python3 -u tools/diag/raft_modes.py raftstereo-sceneflow 1 > gpurun_out/modes_sf_b1.log 2>&1; rc=$?
cat gpurun_out/modes_sf_b1.log | grep -v "^\[I\]" | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u tools/diag/raft_modes.py raftstereo-sceneflow 2 > gpurun_out/modes_sf_b2.log 2>&1; rc=$?
cat gpurun_out/modes_sf_b2.log | grep -v "^\[I\]" | tail -12
exit $rc
