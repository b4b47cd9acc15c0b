set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_crestereo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/agcl_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/agcl_tests.log; [ $rc -eq 0 ] || exit 1
export SA_PLAN_DIR=
for r in 1 2; do for m in crestereo-iter10 crestereo-iter2; do timeout -k 10 200 python -u tools/run_engine.py --model $m --batch 1 --frames 30 2>&1 | grep -v amdgpu.ids | tail -n 1 || exit 1; done; done | tee gpurun_out/agcl_eng.log
NAME=cre10_b1 MODEL=crestereo-iter10 BATCH=1 FRAMES=5 bash tools/gpu/profile_one.sh && grep -i "agcl\|total" gpurun_out/prof_cre10_b1.txt
