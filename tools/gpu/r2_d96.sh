set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "c96 or direct2 or stem" > gpurun_out/d96_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/d96_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes l2b8,l2b1 --cfgs=0,1,4,24 2>&1 | grep -v "amdgpu.ids" > gpurun_out/d96.log && \
timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes l2b8,l2b1 --cfgs=0,24 --stats 16 2>&1 | grep -v "amdgpu.ids" >> gpurun_out/d96.log; cat gpurun_out/d96.log
