#!/bin/bash
# SA_TUNE_LDS_TOL=0.08 restricted to small shapes (SA_TUNE_LDS_MAXM=19200: one 1/4-resolution 480x640 image)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ldstol2; mkdir -p $O
# side-branch convs only (RAFT mode-2 coarse GRU levels)
for m in "raftstereo-realtime 1 30" "crestereo-iter10 1 20" "crestereo-iter5 1 20"; do
  set -- $m
  timeout -k 10 500 python3 tools/ab_engine.py --knob SA_TUNE_LDS_TOL --values 0,0.08 --clear-plan --model $1 --batch $2 --rounds 8 --frames $3 > $O/$1_b$2.log 2>&1 || exit 1
  echo "$1 b$2"; tail -2 $O/$1_b$2.log
done
