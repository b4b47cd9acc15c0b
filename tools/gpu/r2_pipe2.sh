set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 240 python3 -u tools/ab_engine.py --knob SA_RAFT_PIPELINE --values 1,2,0 --model raftstereo-sceneflow --batch 1 --rounds 8 > gpurun_out/pipe2_ab.log 2>&1; r=$?
grep -v "^\[I\]" gpurun_out/pipe2_ab.log | tail -8; [ $r -eq 0 ] || exit $r
timeout -k 10 150 python3 -u tools/diag/replay_stress.py --model raftstereo-sceneflow --reps 16 --rounds 2 --canary 4 2>&1 | grep -v "^\[I\]" | tail -3
timeout -k 10 200 python -u -m pytest tests/test_raft_engine_gpu.py tests/test_fullconfig_gpu.py -q -x -k "sceneflow" --timeout 150 --timeout-method thread 2>&1 | tail -3
