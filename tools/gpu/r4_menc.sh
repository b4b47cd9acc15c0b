#!/bin/bash
# Round 4 motion-encoder / mode-2 layout check (run under gpurun): schedule equality, the layout A/B at b1 / b8,
# and the fused motion encoder's stage stamps for the round-3 kernel (exp lib) vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/menc
timeout -k 10 400 python3 -u -m pytest tests/test_raft_modes_gpu.py -v -rfE --timeout 300 --timeout-method thread > gpurun_out/menc/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/menc/pytest.log
for b in 1 8; do
  timeout -k 10 120 python3 -u tools/diag/menc_stamps.py --batch $b > gpurun_out/menc/stamps_head_b$b.log 2>&1 || exit 1
  SA_NATIVE_LIB=$PWD/stereoalgorithms_amd/lib/exp/libstereo_amd_menc_r3.so timeout -k 10 120 python3 -u tools/diag/menc_stamps.py --batch $b > gpurun_out/menc/stamps_r3_b$b.log 2>&1 || exit 1
done
tail -12 gpurun_out/menc/stamps_r3_b1.log gpurun_out/menc/stamps_head_b1.log gpurun_out/menc/stamps_r3_b8.log gpurun_out/menc/stamps_head_b8.log
timeout -k 10 300 python3 -u tools/ab_engine.py --knob SA_RAFT_M2_MAIN --values 0,1 --batch 1 --rounds 5 > gpurun_out/menc/ab_b1.log 2>&1 && tail -2 gpurun_out/menc/ab_b1.log &&
timeout -k 10 400 python3 -u tools/ab_engine.py --knob SA_RAFT_M2_MAIN --values 0,1 --batch 8 --rounds 4 > gpurun_out/menc/ab_b8.log 2>&1 && tail -2 gpurun_out/menc/ab_b8.log
