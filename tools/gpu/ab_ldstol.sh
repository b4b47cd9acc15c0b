#!/bin/bash
# Tuner LDS-footprint tie-break (SA_TUNE_LDS_TOL) A/B: each engine tunes fresh in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ldstol; mkdir -p $O
for m in "raftstereo-sceneflow 1 20" "raftstereo-realtime 1 30" "crestereo-iter10 1 20" "raftstereo-sceneflow 8 5"; do
  set -- $m
  timeout -k 10 500 python3 tools/ab_engine.py --knob SA_TUNE_LDS_TOL --values 0,0.08,0.2 --clear-plan --model $1 --batch $2 --rounds 6 --frames $3 > $O/$1_b$2.log 2>&1 || exit 1
  echo "$1 b$2"; tail -3 $O/$1_b$2.log
done
