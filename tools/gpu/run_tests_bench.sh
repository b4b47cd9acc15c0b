set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1 && echo BENCH_OK
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench1.log
