#!/bin/bash
# conv kernel numerics + A/B micro-benchmark (run under gpurun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
timeout -k 10 300 python3 -u tools/conv_bench.py --cfgs=${CFGS:--1,4} --shapes ${SHAPES:-zr8,q8,fh8,enc8,l1b8,zr8s,zr1,q1} > gpurun_out/conv_bench.log 2>&1
cat gpurun_out/conv_bench.log
