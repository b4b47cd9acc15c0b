set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "glds3" -q --timeout 100 --timeout-method thread > gpurun_out/wide_ops.log 2>&1
rc=$?; tail -3 gpurun_out/wide_ops.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/conv_bench.py --iters 30 --shapes zr8,q8,fh8,enc8,zr8s --cfgs 4,7,10,11 > gpurun_out/cb.log 2>&1; cat gpurun_out/cb.log | grep cfg
SHAPES=zr8,q8 CFGS=4,10,11 bash tools/gpu/pmc_conv.sh > /dev/null 2>&1; grep -E "kernel|MFMA busy|TCC_MISS|TCC_HIT" gpurun_out/pmc_a.txt gpurun_out/pmc_c.txt
