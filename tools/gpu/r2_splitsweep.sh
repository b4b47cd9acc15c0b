set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/conv_bench.py --iters 30 --shapes zr8l,zr32,zr1,q1,fh1,enc1,mc1 --cfgs 3,4,5,7,8 --splits 1,2,4,8 > gpurun_out/splitsweep.log 2>&1
r=$?; grep -v "^\[" gpurun_out/splitsweep.log | tail -150; exit $r
