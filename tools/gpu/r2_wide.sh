set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "glds3" -v --timeout 100 --timeout-method thread > gpurun_out/wide_ops.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error" gpurun_out/wide_ops.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_fullconfig_gpu.py -k "raft" -v -s --timeout 200 --timeout-method thread > gpurun_out/wide_full.log 2>&1
rc=$?
grep -E "PASS|FAIL|^raft|cfg 1[01]" gpurun_out/wide_full.log | tail -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-latency > gpurun_out/bench_w.log 2>&1
tail -c 700 gpurun_out/bench_w.log
