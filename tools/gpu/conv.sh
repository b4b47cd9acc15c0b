#!/bin/bash
# Conv kernel check under gpurun: optional pytest selection, then tools/conv_bench.py over tile configs, optionally
# once per experimental library (tools/exp_build.sh <name> [-D...] builds stereoalgorithms_amd/lib/exp/
# libstereo_amd_<name>.so; list them in LIBS -- and un-ignore lib/exp in .gpurunignore for that call).
#   TESTS="tests/test_ops_gpu.py -k halo" SHAPES=zr8,q8 CFGS=28,32 SPLITS=1,0 LIBS="base nodma" bash tools/gpu/conv.sh tag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-conv}
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python3 -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
ARGS="--graph --iters ${ITERS:-20} --shapes ${SHAPES:-zr8,q8,fh8} --cfgs=${CFGS:--1}"
[ -n "$SPLITS" ] && ARGS="$ARGS --splits $SPLITS"
: > gpurun_out/$T/bench.txt
for v in ${LIBS:-default}; do
  echo "== $v" >> gpurun_out/$T/bench.txt
  if [ "$v" = default ]; then
    timeout -k 10 200 python3 tools/conv_bench.py $ARGS >> gpurun_out/$T/bench.txt 2>&1 || exit 1
  else
    SA_NATIVE_LIB=$PWD/stereoalgorithms_amd/lib/exp/libstereo_amd_$v.so timeout -k 10 200 \
      python3 tools/conv_bench.py $ARGS >> gpurun_out/$T/bench.txt 2>&1 || exit 1
  fi
done
grep -v amdgpu.ids gpurun_out/$T/bench.txt
if [ -n "$PMC" ]; then
  SHAPES=${SHAPES%%,*} CFGS=$CFGS bash tools/gpu/pmc_conv.sh > gpurun_out/$T/pmc.txt 2>&1
  cat gpurun_out/$T/pmc.txt
fi
