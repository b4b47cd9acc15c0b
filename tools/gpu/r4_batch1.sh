#!/bin/bash
# Round-4 batch of checks (run under gpurun): CREStereo tests + parallel-branch A/B, conv tile bench + PMC of the
# halo tiles on the batch-8 GRU shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; O=gpurun_out/b1; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_crestereo_gpu.py tests/test_fullconfig_gpu.py::test_crestereo_iter10_full_config -v -rfEP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|b1: \|ref" $O/pytest.log | tail -4
timeout -k 10 300 python3 -u tools/ab_engine.py --knob SA_CRE_PARALLEL --values 0,1 --model crestereo-iter10 --batch 1 --rounds 5 > $O/ab_cre.log 2>&1 && tail -2 $O/ab_cre.log || exit 1
timeout -k 10 200 python3 tools/conv_bench.py --iters 20 --shapes zr8,q8,fh8,zr8s --cfgs 4,26,27,10 > $O/cb.log 2>&1 && grep -v amdgpu $O/cb.log | tail -18 || exit 1
SHAPES=zr8 CFGS=26,27 bash tools/gpu/pmc_conv.sh > $O/pmc_halo.txt 2>&1; echo "pmc rc=$?"
