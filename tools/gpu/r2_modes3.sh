set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 300 python3 -u tools/diag/raft_modes.py raftstereo-sceneflow 1 > gpurun_out/modes3_sf_b1.log 2>&1; rc=$?
grep -v "^\[I\]" gpurun_out/modes3_sf_b1.log | tail -9; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u tools/ab_engine.py --knob SA_RAFT_PIPELINE --values 1,2 --model raftstereo-sceneflow --batch 1 --rounds 8 > gpurun_out/pipe2_ab.log 2>&1; r=$?
grep -v "^\[I\]" gpurun_out/pipe2_ab.log | tail -3
