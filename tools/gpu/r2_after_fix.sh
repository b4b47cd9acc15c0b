set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
export SA_PLAN_DIR=/tmp/sa_plans
LOG=gpurun_out/stress_all.log
: > $LOG
for m in raftstereo-sceneflow raftstereo-realtime crestereo-iter2 crestereo-iter5 crestereo-iter10 hitnet-d400 hitnet-xl fastacvnet-plus; do
  timeout -k 10 150 python3 -u tools/diag/replay_stress.py --model $m --reps 16 --rounds 2 --canary 4 2>&1 | grep TOTAL >> $LOG
  r=$?; [ $r -gt 1 ] && { cat $LOG; exit $r; }
done
cat $LOG
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1 && echo BENCH_OK
tail -c 600 gpurun_out/bench1.log
