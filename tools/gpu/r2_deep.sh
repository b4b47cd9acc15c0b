set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "glds3_vs_torch or streamk" -x -q --timeout 120 --timeout-method thread > gpurun_out/deep_test.log 2>&1
rc=$?
tail -5 gpurun_out/deep_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/conv_bench.py --iters 30 --shapes zr8l,zr32,zr1,q1,fh1,enc1,mc1,zr8,q8,fh8,enc8 --cfgs 4,5,7,14,15,16,17 --splits 1,0 > gpurun_out/deep_bench.log 2>&1
r=$?; grep -v "^\[" gpurun_out/deep_bench.log | tail -5; exit $r
