# HITNet warp cost: one thread per (candidate, tile pixel) vs per (candidate, tile) (SA_HIT_WARP_PX), b1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hitnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hw_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/hw_tests.log; [ $rc -eq 0 ] || exit 1
for m in hitnet-d400 hitnet-xl; do timeout -k 10 300 python -u tools/ab_engine.py --knob SA_HIT_WARP_PX --values 0,1 --model $m --batch 1 --rounds 7 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/hw_ab.log
