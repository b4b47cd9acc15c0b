set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/conv_bench.py --iters 30 --gemm-ref 1 --shapes zr8,q8,fh8,zr8g,q8g --cfgs=-1,4,7,10 > gpurun_out/ceiling.log 2>&1 && cat gpurun_out/ceiling.log
