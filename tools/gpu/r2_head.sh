# HEAD check after a container rebuild: full GPU suite, then the driver's default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_head.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_head.log
[ $rc -eq 0 ] && timeout -k 10 300 python -u bench.py > gpurun_out/bench_head.log 2>&1 && tail -c 600 gpurun_out/bench_head.log
