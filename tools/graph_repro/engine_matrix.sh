#!/bin/bash
# The engine's own graph-replay screens under each packet-capture / stream-kind setting (one process each;
# the runtime reads DEBUG_CLR_GRAPH_PACKET_CAPTURE at initialisation), then frame latency on vs off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T="tests/test_raft_engine_gpu.py::test_engine_cloud_and_rectify_roundtrip tests/test_raft_engine_gpu.py::test_replay_determinism_race_screen tests/test_parallel_gpu.py"
for pc in 1 0; do
  for nb in 0 1; do
    echo "== packet_capture=$pc engine_stream_blocking=$nb"
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc SA_ENGINE_STREAM_BLOCKING=$nb timeout -k 10 200 \
      python -u -m pytest $T -q --timeout 100 --timeout-method thread 2>&1 | tail -2
    r=$?; [ $r -gt 1 ] && exit $r
  done
done
for pc in 1 0; do
  echo "== latency packet_capture=$pc"
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 200 python -u tools/graph_repro/latency.py || exit 1
done
