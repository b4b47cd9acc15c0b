set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 600 python -u -m pytest tests/test_plan_cache_gpu.py tests/test_fullconfig_gpu.py tests/test_raft_engine_gpu.py tests/test_crestereo_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r2b.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|device bytes|plan|^(raft|cre|fast|mean)" gpurun_out/r2b.log | grep -v "^  cfg" | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-latency > gpurun_out/bench_b.log 2>&1
tail -c 900 gpurun_out/bench_b.log
