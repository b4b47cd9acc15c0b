#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/hs; mkdir -p $O
timeout -k 10 400 python3 tools/ab_engine.py --knob SA_TUNE_HALO_SPLIT --values 0,1 --clear-plan --model raftstereo-sceneflow --batch 8 --rounds 4 > $O/sf8.log 2>&1 || exit 1
tail -4 $O/sf8.log
timeout -k 10 300 python3 tools/ab_engine.py --knob SA_TUNE_HALO_SPLIT --values 0,1 --clear-plan --model raftstereo-sceneflow --batch 1 --rounds 6 --frames 20 > $O/sf1.log 2>&1 || exit 1
tail -4 $O/sf1.log
timeout -k 10 300 python3 tools/ab_engine.py --knob SA_TUNE_HALO_SPLIT --values 0,1 --clear-plan --model crestereo-iter10 --batch 1 --rounds 6 --frames 20 > $O/cre.log 2>&1 || exit 1
tail -4 $O/cre.log
