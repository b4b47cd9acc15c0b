#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ldstol3; mkdir -p $O
for m in "hitnet-d400 1 30" "fastacvnet-plus 1 30"; do
  set -- $m
  timeout -k 10 500 python3 tools/ab_engine.py --knob SA_TUNE_LDS_TOL --values 0,0.08 --clear-plan --model $1 --batch $2 --rounds 8 --frames $3 > $O/$1.log 2>&1 || exit 1
  echo "$1"; tail -2 $O/$1.log
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_hitnet_gpu.py tests/test_fast_acvnet_gpu.py > $O/pytest.log 2>&1; tail -1 $O/pytest.log
