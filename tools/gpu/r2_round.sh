# HEAD: full GPU suite, driver bench, RAFT-SF kernel profiles (b1, b8, b8 serialized)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_round.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_gpu_round.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_round.log 2>&1 || exit 1
tail -c 300 gpurun_out/bench_round.log
run() { NAME=$1 MODEL=$2 BATCH=$3 FRAMES=$4 bash tools/gpu/profile_one.sh || return 1; }
run sf_b1 raftstereo-sceneflow 1 5 && run sf_b8 raftstereo-sceneflow 8 3 && \
SA_RAFT_PARALLEL=0 run sf_b8_serial raftstereo-sceneflow 8 3 && run rt_b1 raftstereo-realtime 1 10
for f in gpurun_out/prof_*.txt; do echo "== $f"; head -n 2 $f; done
