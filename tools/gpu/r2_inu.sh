set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "norm" > gpurun_out/inu_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/inu_tests.log; [ $rc -eq 0 ] || exit 1
for b in 1 8; do timeout -k 10 300 python -u tools/ab_engine.py --knob SA_IN_UNROLL --values 4,8 --batch $b --rounds 7 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/inu_ab.log
