# HEAD health (GPU suite + bench) and the GEMM ceiling reference for the RAFT hot conv shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log && \
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1 && echo BENCH_OK && \
timeout -k 10 200 python -u tools/conv_bench.py --iters 30 --gemm-ref 1 --shapes zr8,q8,fh8,zr8g,q8g --cfgs=-1,4,7,10 > gpurun_out/ceiling.log 2>&1 && cat gpurun_out/ceiling.log
