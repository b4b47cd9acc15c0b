set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_crestereo_gpu.py tests/test_fullconfig_gpu.py -x -q -k "linear or crestereo" --timeout 200 --timeout-method thread > gpurun_out/la_tests.log 2>&1
rc=$?; tail -3 gpurun_out/la_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/run_engine.py --model crestereo-iter10 --batch 1 --frames 20 2>&1 | grep -v "^\[I\]\|amdgpu" | tail -2
timeout -k 10 200 python3 -u tools/run_engine.py --model crestereo-iter2 --batch 1 --frames 20 2>&1 | grep -v "^\[I\]\|amdgpu" | tail -2
