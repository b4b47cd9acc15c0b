cd $GRAFT_REPO_ROOT
for v in base NODMA NOMFMA NOLDSREAD NOBAR NODMA_NOBAR ONLYMFMA; do
  if [ $v = base ]; then unset SA_NATIVE_LIB; else export SA_NATIVE_LIB=$PWD/stereoalgorithms_amd/lib/exp/libstereo_amd_$v.so; fi
  echo "== $v"
  timeout -k 5 60 python -u tools/conv_bench.py --iters 20 --shapes zr8,zr8s --cfgs 10 2>&1 | grep cfg || exit 1
done
