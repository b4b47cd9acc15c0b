set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in raftstereo-sceneflow raftstereo-realtime; do timeout -k 10 300 python -u tools/ab_engine.py --knob SA_CORR_SPLIT --values 0,1 --model $m --batch 1 --rounds 7 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/corr_ab.log
