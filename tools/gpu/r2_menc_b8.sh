set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_engine.py --knob SA_RAFT_FUSE_MENC --values 1,0 --batch 8 --rounds 5 2>&1 | grep -v "amdgpu.ids\|^\[I\]" | tee gpurun_out/menc_b8.log
timeout -k 10 400 python -u tools/ab_engine.py --knob SA_RAFT_FUSE_FH --values 0,1 --batch 8 --rounds 5 2>&1 | grep -v "amdgpu.ids\|^\[I\]" | tee -a gpurun_out/menc_b8.log
