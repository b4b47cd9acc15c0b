set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 100 python -u tools/diag/inn_determinism.py 2>&1 | grep -v amdgpu.ids
SA_FUSE_IN=0 timeout -k 10 200 python -u -m pytest tests/test_raft_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "matches_oracle" 2>&1 | tail -n 2
