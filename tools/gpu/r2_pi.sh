set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_raft_engine_gpu.py tests/test_raft_modes_gpu.py -x -q --timeout 120 --timeout-method thread -k "pool or interp or raft" > gpurun_out/pi_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/pi_tests.log; [ $rc -eq 0 ] || exit 1
for b in 1 8; do timeout -k 10 300 python -u tools/ab_engine.py --knob SA_RAFT_POOL_INTERP --values 0,1 --batch $b --rounds 5 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/pi_ab.log
