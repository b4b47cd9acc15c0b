# direct conv v2 with contiguous tile runs per workgroup: tests + bench (with / without statistics)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "direct" > gpurun_out/d2b_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/d2b_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes fr8,fnet,mc1s1 --cfgs=9,23 2>&1 | grep -v amdgpu.ids > gpurun_out/d2b.log && \
timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes fr8,fnet --cfgs=9,23 --stats 16 2>&1 | grep -v amdgpu.ids >> gpurun_out/d2b.log && cat gpurun_out/d2b.log
