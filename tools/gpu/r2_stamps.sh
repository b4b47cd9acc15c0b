set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 100 python3 -u tools/diag/menc_stamps.py --batch 1 --waves 4 2>&1 | grep -v "^\[I\]\|amdgpu.ids" && \
timeout -k 10 100 python3 -u tools/diag/menc_stamps.py --batch 8 --waves 4 2>&1 | grep -v "^\[I\]\|amdgpu.ids" && \
timeout -k 10 100 python3 -u tools/diag/menc_stamps.py --batch 8 --waves 8 2>&1 | grep -v "^\[I\]\|amdgpu.ids"
