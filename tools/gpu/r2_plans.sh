# per-shape tuned conv times (plan files) and device stage stamps, RAFT-SF b8 / b1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SA_PLAN_CACHE=gpurun_out/plan_sf_b8.txt
rm -f $SA_PLAN_CACHE
timeout -k 10 200 python -u tools/run_engine.py --model raftstereo-sceneflow --batch 8 --frames 10 > gpurun_out/stages_sf_b8.log 2>&1 && \
SA_PLAN_CACHE=gpurun_out/plan_sf_b1.txt timeout -k 10 200 python -u tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 20 > gpurun_out/stages_sf_b1.log 2>&1 && \
SA_RAFT_PARALLEL=0 SA_RAFT_PIPELINE=0 SA_PLAN_CACHE=gpurun_out/plan_sf_b8.txt timeout -k 10 200 python -u tools/run_engine.py --model raftstereo-sceneflow --batch 8 --frames 10 > gpurun_out/stages_sf_b8_serial.log 2>&1
tail -2 gpurun_out/stages_sf_b8.log gpurun_out/stages_sf_b1.log gpurun_out/stages_sf_b8_serial.log
