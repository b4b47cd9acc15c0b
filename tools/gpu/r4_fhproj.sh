#!/bin/bash
# Flow-head tap projection fused into conv1's epilogue: op test + RAFT engine tests, then same-process A/B
# (SA_RAFT_FH_PROJ) at b1 / b8 and the realtime preset; then the side-branch marks of RT / CREStereo (SA_TUNE_LDS_TOL)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/fhp; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "tap_projection or flow_acc" tests/test_raft_engine_gpu.py tests/test_crestereo_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in "raftstereo-sceneflow 1 20" "raftstereo-sceneflow 8 5" "raftstereo-realtime 1 30"; do
  set -- $m
  timeout -k 10 500 python3 tools/ab_engine.py --knob SA_RAFT_FH_PROJ --values 0,1 --model $1 --batch $2 --rounds 6 --frames $3 > $O/$1_b$2.log 2>&1 || exit 1
  echo "FH_PROJ $1 b$2"; tail -2 $O/$1_b$2.log
done
timeout -k 10 500 python3 tools/ab_engine.py --knob SA_CRE_FH_PROJ --values 0,1 --model crestereo-iter10 --batch 1 --rounds 6 --frames 20 > $O/cre.log 2>&1 || exit 1
echo "FH_PROJ crestereo-iter10"; tail -2 $O/cre.log
for m in "raftstereo-realtime 1 30" "crestereo-iter10 1 20"; do
  set -- $m
  timeout -k 10 500 python3 tools/ab_engine.py --knob SA_TUNE_LDS_TOL --values 0,0.08 --clear-plan --model $1 --batch $2 --rounds 6 --frames $3 > $O/lds_$1_b$2.log 2>&1 || exit 1
  echo "LDS_TOL $1 b$2"; tail -2 $O/lds_$1_b$2.log
done
