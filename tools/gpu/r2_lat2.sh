set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_demos_gpu.py tests/test_raft_engine_gpu.py tests/test_plan_cache_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lat2_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/lat2_tests.log; [ $rc -eq 0 ] || exit 1
for m in raftstereo-realtime raftstereo-sceneflow; do timeout -k 10 200 python -u tools/diag/latency_parts.py --model $m --frames 30 2>&1 | grep -v "amdgpu.ids\|^\[I\]" || exit 1; done | tee gpurun_out/lat_parts2.log
