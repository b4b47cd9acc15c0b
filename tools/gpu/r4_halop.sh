#!/bin/bash
# Planar halo tiles (cfg 28/29): numerics vs torch, micro-bench against the swizzled ones (26/27), PMC of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; O=gpurun_out/hp; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -k "halo" -v -rfE --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
prc=$?; echo "pytest rc=$prc"; grep -E "passed|failed" $O/pytest.log | tail -3
[ $prc -le 1 ] || exit $prc
timeout -k 10 200 python3 tools/conv_bench.py --iters 20 --shapes zr8,q8,fh8,zr8s,zr1,q1,fh1,zr8l --cfgs 26,27,28,29 > $O/cb.log 2>&1 && grep -v amdgpu $O/cb.log | tail -32 || exit 1
SHAPES=zr8 CFGS=27,29 bash tools/gpu/pmc_conv.sh > $O/pmc.txt 2>&1; echo "pmc rc=$?"
