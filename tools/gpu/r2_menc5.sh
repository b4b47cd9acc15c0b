set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_raft_modes_gpu.py tests/test_raft_engine_gpu.py tests/test_fullconfig_gpu.py tests/test_replay_stress_gpu.py -x -q -k "motion or corr or raft or schedules or replays" --timeout 200 --timeout-method thread > gpurun_out/menc5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/menc5_tests.log; [ $rc -eq 0 ] || exit $rc
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 240 python3 -u tools/ab_engine.py --knob SA_RAFT_FUSE_MENC --values 0,1 --model raftstereo-sceneflow --batch 8 --rounds 6 > gpurun_out/menc_ab8.log 2>&1; r=$?
grep -v "^\[I\]" gpurun_out/menc_ab8.log | tail -3; [ $r -eq 0 ] || exit $r
timeout -k 10 240 python3 -u tools/ab_engine.py --knob SA_RAFT_FUSE_MENC --values 0,1 --model raftstereo-realtime --batch 1 --rounds 8 > gpurun_out/menc_ab_rt.log 2>&1; r=$?
grep -v "^\[I\]" gpurun_out/menc_ab_rt.log | tail -3
