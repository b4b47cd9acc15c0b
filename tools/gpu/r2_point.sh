set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "point or conv2d_vs_torch" > gpurun_out/point_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/point_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes ds8,ds1,ds38 --cfgs=0,1,11,25 2>&1 | grep -v "amdgpu.ids\|rc=-5" > gpurun_out/point.log && \
timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes ds8,ds38 --cfgs=1,11,25 --stats 16 2>&1 | grep -v "amdgpu.ids\|rc=-5" >> gpurun_out/point.log; cat gpurun_out/point.log
for cfg in "raftstereo-sceneflow 8 10" "raftstereo-sceneflow 1 20"; do set -- $cfg
  SA_PLAN_CACHE=gpurun_out/plan_${1}_b$2.txt timeout -k 10 200 python -u tools/run_engine.py --model $1 --batch $2 --frames $3 2>&1 | grep -v amdgpu.ids | tail -n 1 || exit 1
done
