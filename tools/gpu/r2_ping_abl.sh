# ablation builds of the ping-pong schedule (results of NO* variants are garbage: timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base nodma nobar nolds nomfma; do
  SA_NATIVE_LIB=stereoalgorithms_amd/lib/exp/libstereo_amd_$v.so timeout -k 10 100 python -u tools/conv_bench.py --iters 30 --shapes zr8,q8 --cfgs=18,19 --splits=1 > gpurun_out/abl_$v.log 2>&1 || exit 1
  echo "== $v"; grep cfg gpurun_out/abl_$v.log
done
