# ping-pong conv tiles: op tests, then the RAFT hot shapes against the current tactics
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "glds3 or ping or projection" > gpurun_out/ping_tests.log 2>&1; rc=$?; tail -5 gpurun_out/ping_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 200 python -u tools/conv_bench.py --iters 30 --shapes zr8,q8,fh8,enc8,zr1,q1,fh1 --cfgs=4,7,18,19 --splits=1,0 > gpurun_out/ping_bench.log 2>&1 && cat gpurun_out/ping_bench.log
