set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_raft_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "corr or matches_oracle" > gpurun_out/corr_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/corr_tests.log; [ $rc -eq 0 ] || exit 1
export SA_PLAN_DIR=
for r in 1 2; do for cfg in "raftstereo-sceneflow 1 20" "raftstereo-realtime 1 30"; do set -- $cfg
  timeout -k 10 200 python -u tools/run_engine.py --model $1 --batch $2 --frames $3 2>&1 | grep -v amdgpu.ids | tail -n 1 || exit 1
done; done | tee gpurun_out/corr_eng.log
