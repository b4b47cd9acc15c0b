# Fast-ACVNet+ kernel A/Bs (depthwise 3x3 SA_DWCONV_LDS, correlation volume SA_NORM_CORR8, concat volume SA_CONCAT_CHUNK), b1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fast_acvnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dw_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/dw_tests.log; [ $rc -eq 0 ] || exit 1
SA_CONCAT_CHUNK=1 timeout -k 10 300 python -u -m pytest tests/test_fast_acvnet_gpu.py -x -q --timeout 120 --timeout-method thread -k "dwconv or norm_corr or concat" 2>&1 | tail -n 1
timeout -k 10 300 python -u tools/ab_engine.py --knob SA_CONCAT_CHUNK --values 0,1 --model fastacvnet-plus --batch 1 --rounds 7 2>&1 | grep -v "amdgpu.ids\|^\[I\]" | tee gpurun_out/cc_ab.log
