#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/prio; mkdir -p $O
export SA_PLAN_DIR=/tmp/sa_plans
for m in "raftstereo-sceneflow 1 20" "raftstereo-realtime 1 30" "crestereo-iter10 1 20" "raftstereo-sceneflow 8 5"; do
  set -- $m
  timeout -k 10 400 python3 tools/ab_engine.py --knob SA_STREAM_PRIO --values 0,1 --model $1 --batch $2 --rounds 6 --frames $3 > $O/$1_b$2.log 2>&1 || exit 1
  echo "$1 b$2"; tail -2 $O/$1_b$2.log
done
