set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sx
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -k "workgroup_splitk or gru_zrq_split" > gpurun_out/sx/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/sx/pytest.log; exit 1; }
tail -3 gpurun_out/sx/pytest.log
timeout -k 10 300 python3 -u tools/conv_bench.py --shapes zr32,q32,zr8l,q8l --cfgs=-1,16,14,37,38 --splits 1 > gpurun_out/sx/conv_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/sx/conv_bench.log; exit 1; }
cat gpurun_out/sx/conv_bench.log | grep -v amdgpu.ids
