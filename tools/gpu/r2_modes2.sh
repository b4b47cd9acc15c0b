set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 300 python3 -u tools/diag/raft_modes.py raftstereo-sceneflow 1 > gpurun_out/modes2_sf_b1.log 2>&1; rc=$?
grep -v "^\[I\]" gpurun_out/modes2_sf_b1.log | tail -12
exit $rc
