set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base ns5 base ns5; do
  SA_NATIVE_LIB=stereoalgorithms_amd/lib/exp/libstereo_amd_$v.so timeout -k 10 100 python -u tools/conv_bench.py --iters 50 --shapes zr8,zr1 --cfgs=4,18 --splits=1,0 > gpurun_out/ns_$v.log 2>&1 || exit 1
  echo "== $v"; grep cfg gpurun_out/ns_$v.log
done
