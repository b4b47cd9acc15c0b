set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 300 python -u -m pytest tests/test_fullconfig_gpu.py -k raft -q --timeout 200 --timeout-method thread > gpurun_out/cf2.log 2>&1; tail -2 gpurun_out/cf2.log
timeout -k 10 300 python3 tools/ab_engine.py --knob SA_RAFT_MERGE_CF2 --values 1,0 --batch 1 --rounds 4 --frames 20 2>&1 | grep SA_
timeout -k 10 300 python3 tools/ab_engine.py --knob SA_RAFT_MERGE_CF2 --values 1,0 --batch 8 --rounds 4 --frames 4 2>&1 | grep SA_
