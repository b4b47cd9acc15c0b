set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_raft_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "direct2 or matches_oracle" > gpurun_out/inn3_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/inn3_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 100 python -u tools/diag/inn_determinism.py 2>&1 | grep -v amdgpu.ids | tail -n 2
for b in 8 1; do timeout -k 10 300 python -u tools/ab_engine.py --knob SA_FUSE_IN --values 0,1 --batch $b --rounds 5 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/inn3_ab.log
