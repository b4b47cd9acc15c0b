set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/split_batch_ab.py --batch 8 --splits 1,2,4 --rounds 3 --steps 10 2>&1 | grep -v "amdgpu.ids\|^\[I\]" | tee gpurun_out/split_ab.log
