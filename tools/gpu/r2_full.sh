# full GPU suite + bench at the working tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1 && echo BENCH_OK && python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/bench1.log') if x.startswith('{')][-1]; d=json.loads(l)
print({k:d[k] for k in ['value','ms_per_step','vs_baseline']}); print({k:(v['latency_ms_p50']) for k,v in d['latency_b1'].items()})
PY
