#!/bin/bash
# Driver-shaped check (run under gpurun): the default bench.py line exactly as the round-end driver runs it (its exit
# status matters), then the whole GPU test suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
T=${1:-r3e}
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/tl/${T}_bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "bench rc=0"; tail -1 gpurun_out/tl/${T}_bench.log | cut -c1-400
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tl/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/tl/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/tl/${T}_pytest.log
