set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -k "motion" -x -q --timeout 120 --timeout-method thread > gpurun_out/menc_test.log 2>&1
rc=$?; tail -3 gpurun_out/menc_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python3 -u tools/diag/menc_stamps.py --batch 1 --waves 4 2>&1 | grep -v "^\[I\]\|amdgpu.ids" && \
timeout -k 10 100 python3 -u tools/diag/menc_stamps.py --batch 8 --waves 4 2>&1 | grep -v "^\[I\]\|amdgpu.ids" && \
timeout -k 10 100 python3 -u tools/diag/menc_stamps.py --batch 8 --waves 8 2>&1 | grep -v "^\[I\]\|amdgpu.ids" || exit 1
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 240 python3 -u tools/ab_engine.py --knob SA_RAFT_FUSE_MENC --values 0,1 --model raftstereo-sceneflow --batch 8 --rounds 6 > gpurun_out/menc_ab8.log 2>&1; r=$?
grep -v "^\[I\]" gpurun_out/menc_ab8.log | tail -3; [ $r -eq 0 ] || exit $r
timeout -k 10 240 python3 -u tools/ab_engine.py --knob SA_RAFT_FUSE_MENC --values 0,1 --model raftstereo-sceneflow --batch 1 --rounds 8 > gpurun_out/menc_ab1.log 2>&1; r=$?
grep -v "^\[I\]" gpurun_out/menc_ab1.log | tail -3
