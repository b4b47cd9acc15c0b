# 7x7 stem kernel: op tests + bench vs the implicit GEMM; direct 3x3 c64 ablations on the full-res shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem or direct" > gpurun_out/stem_tests.log 2>&1; rc=$?; tail -n 5 gpurun_out/stem_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 200 python -u tools/conv_bench.py --iters 20 --shapes stem1,stem8,stemrt --cfgs=1,0,22 > gpurun_out/stem_bench.log 2>&1 && cat gpurun_out/stem_bench.log && \
for abl in 0 1 2 4 8 16 6; do SA_DIRECT_ABL=$abl timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes fr8,fnet --cfgs=9 2>&1 | grep -v amdgpu.ids | sed "s/^/abl$abl /" || exit 1; done > gpurun_out/direct_abl.log && cat gpurun_out/direct_abl.log
