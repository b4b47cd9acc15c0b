set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 0 2; do
SA_RAFT_PIPELINE=$m SA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearse_w2_p$m.log 2>&1 || { tail -n 20 gpurun_out/rehearse_w2_p$m.log; exit 1; }
grep '^{' gpurun_out/rehearse_w2_p$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w2 gloo pipeline $m', d['n_gpus'], d['value'], d['ms_per_step'], d.get('allgather_ms'))"
done
