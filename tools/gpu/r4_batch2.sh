#!/bin/bash
# Round-4 batch 2 (run under gpurun): CREStereo tests, A/Bs of the CREStereo context precompute, the realtime fused
# motion encoder at batch 1, and the wide-tile grid threshold at batch 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; O=gpurun_out/b2; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_crestereo_gpu.py tests/test_fullconfig_gpu.py::test_crestereo_iter10_full_config -v -rfEP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|b1: \|ref" $O/pytest.log | tail -3
ab() {  # tag knob values model batch [extra]
  timeout -k 10 400 python3 -u tools/ab_engine.py --knob $2 --values $3 --model $4 --batch $5 --rounds 5 $6 > $O/ab_$1.log 2>&1 || { echo "ab $1 failed"; tail -3 $O/ab_$1.log; return 1; }
  echo "== $1"; grep -v amdgpu $O/ab_$1.log | tail -3
}
ab cre2 SA_CRE_CST 0,1 crestereo-iter2 1 && ab cre10 SA_CRE_CST 0,1 crestereo-iter10 1 &&
ab rtme SA_RAFT_FUSE_MENC 0,1 raftstereo-realtime 1 && ab mt8 SA_TUNE_MIN_TILES 256,128 raftstereo-sceneflow 8 --clear-plan
