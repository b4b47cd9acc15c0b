# multi-rank rehearsal on one GPU: bench.py --gpus 2 self-launch over gloo (two ranks share the device), and the
# native RCCL all-gather path forced at world size 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearse_w2.log 2>&1 || { tail -n 20 gpurun_out/rehearse_w2.log; exit 1; }
grep '^{' gpurun_out/rehearse_w2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w2 gloo', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d.get('world_size'), d.get('allgather_ms'))"
SA_DP_GATHER_WORLD1=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-latency 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w1 rccl gather', d['n_gpus'], d['value'], d['ms_per_step'])"
