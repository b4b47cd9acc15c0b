set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fast_acvnet_gpu.py tests/test_hitnet_gpu.py tests/test_fullconfig_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/small_tests.log 2>&1
rc=$?; tail -3 gpurun_out/small_tests.log; [ $rc -eq 0 ] || exit $rc
for m in fastacvnet-plus hitnet-d400 hitnet-xl; do
  timeout -k 10 200 python3 -u tools/run_engine.py --model $m --batch 1 --frames 30 2>&1 | grep -v "^\[I\]\|amdgpu" | tail -1 || exit 1
done
