# direct conv v2 (cfg 23) tests + bench vs cfg 9 on the full-res encoder shapes (with / without IN stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "direct or stem" > gpurun_out/direct2_tests.log 2>&1; rc=$?; tail -n 5 gpurun_out/direct2_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 200 python -u tools/conv_bench.py --iters 20 --shapes fr8,fnet,mc1s1 --cfgs=9,23 > gpurun_out/direct2_bench.log 2>&1 && \
timeout -k 10 200 python -u tools/conv_bench.py --iters 20 --shapes fr8,fnet --cfgs=9,23 --stats 16 >> gpurun_out/direct2_bench.log 2>&1; cat gpurun_out/direct2_bench.log
