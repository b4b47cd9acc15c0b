# tuner: split-K candidates for the deep DMA rings (SA_TUNE_DEEP_SPLIT), fresh processes, no plan cache
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SA_PLAN_DIR=
for r in 1 2; do for v in 0 1; do for cfg in "raftstereo-realtime 1 30" "raftstereo-sceneflow 1 20"; do set -- $cfg
  SA_TUNE_DEEP_SPLIT=$v timeout -k 10 200 python -u tools/run_engine.py --model $1 --batch $2 --frames $3 2>&1 | grep -v amdgpu.ids | tail -n 1 | sed "s/^/deep_split=$v round $r: /" || exit 1
done; done; done | tee gpurun_out/dsplit.log
