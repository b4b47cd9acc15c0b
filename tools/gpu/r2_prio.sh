set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
: > gpurun_out/prio.log
for v in BASE PRIOHI PRIOLO BASE PRIOHI PRIOLO; do
  echo "== $v" >> gpurun_out/prio.log
  SA_NATIVE_LIB=stereoalgorithms_amd/lib/exp/libstereo_amd_$v.so timeout -k 10 120 python3 -u tools/conv_bench.py --iters 40 --shapes zr8,q8,fh8,enc8,zr1,q1 --cfgs 4,7,10,11 --splits 1 2>&1 | grep -v "^\[" >> gpurun_out/prio.log || exit 1
done
cat gpurun_out/prio.log | tail -5
