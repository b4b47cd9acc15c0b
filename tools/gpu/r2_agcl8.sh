set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_crestereo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/agcl8_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/agcl8_tests.log; [ $rc -eq 0 ] || exit 1
SA_AGCL8=0 timeout -k 10 300 python -u -m pytest tests/test_crestereo_gpu.py -x -q --timeout 120 --timeout-method thread -k agcl 2>&1 | tail -n 1
for m in crestereo-iter10 crestereo-iter2; do timeout -k 10 300 python -u tools/ab_engine.py --knob SA_AGCL8 --values 0,1 --model $m --batch 1 --rounds 7 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/agcl8_ab.log
