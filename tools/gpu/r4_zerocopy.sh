#!/bin/bash
# Zero-copy run_host outputs (pinned buffers written by the frame graph's reprojection): correctness test, then the
# host-overhead table with the blocking wait and with SA_HOST_SPIN=1 (polling wait).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/zc; mkdir -p $O
export SA_PLAN_DIR=/tmp/sa_plans
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_raft_engine_gpu.py -k "cloud_and_rectify" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
SA_HOST_TIMES=1 timeout -k 10 300 python3 -u tools/host_overhead.py --presets raftstereo-realtime,hitnet-d400,fastacvnet-plus > $O/block.jsonl 2>$O/block.err || exit 1
cat $O/block.jsonl
SA_HOST_SPIN=1 SA_HOST_TIMES=1 timeout -k 10 300 python3 -u tools/host_overhead.py --presets raftstereo-realtime,hitnet-d400,fastacvnet-plus > $O/spin.jsonl 2>$O/spin.err || exit 1
cat $O/spin.jsonl
