set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/zrq2
timeout -k 10 300 python3 -u tools/ab_engine.py --knob SA_RAFT_ZRQ_PARTS --values 0,1,2 --model raftstereo-sceneflow --batch 1 --rounds 4 > gpurun_out/zrq2/ab_par.log 2>&1 && tail -3 gpurun_out/zrq2/ab_par.log &&
SA_RAFT_PARALLEL=0 timeout -k 10 300 python3 -u tools/ab_engine.py --knob SA_RAFT_ZRQ_PARTS --values 0,1 --model raftstereo-sceneflow --batch 1 --rounds 4 > gpurun_out/zrq2/ab_ser.log 2>&1 && tail -2 gpurun_out/zrq2/ab_ser.log &&
export SA_PLAN_CACHE=/tmp/p.txt SA_RAFT_ZRQ_PARTS=1 && timeout -k 10 120 python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 3 > /dev/null 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d /tmp/tlz -o run -- python3 tools/run_engine.py --model raftstereo-sceneflow --batch 1 --frames 4 > gpurun_out/zrq2/prof.log 2>&1 &&
python3 tools/timeline.py /tmp/tlz --iter-marker motion_encoder --chain 40 > gpurun_out/zrq2/tl_parts1.txt 2>&1
