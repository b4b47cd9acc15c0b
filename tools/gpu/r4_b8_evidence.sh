#!/bin/bash
# b8 evidence at HEAD (run under gpurun): the sceneflow step's kernel profile (default multi-stream schedule and one
# serialized stream), then one PMC pass over a serialized b8 frame: MFMA busy cycles, busy / wave / wait cycles and
# the clock counter per kernel (tools/pmc_summary.py derives the MFMA busy fraction).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ev8; mkdir -p $O
NAME=sf_b8 MODEL=raftstereo-sceneflow BATCH=8 FRAMES=3 bash tools/gpu/profile_one.sh || exit 1
NAME=sf_b8_serial MODEL=raftstereo-sceneflow BATCH=8 FRAMES=3 SA_RAFT_PARALLEL=0 SA_RAFT_PIPELINE=0 bash tools/gpu/profile_one.sh || exit 1
cp gpurun_out/prof_sf_b8.txt gpurun_out/prof_sf_b8_serial.txt $O/
# PMC: reuse the serialized profile's tuned plan; 1 frame
export SA_PLAN_CACHE=/tmp/sa_plan_sf_b8_serial.txt
rm -rf /tmp/pmc8
SA_RAFT_PARALLEL=0 SA_RAFT_PIPELINE=0 timeout -s KILL 150 rocprofv3 --output-format csv \
  --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  -d /tmp/pmc8 -o run -- python3 tools/run_engine.py --model raftstereo-sceneflow --batch 8 --frames 1 > $O/pmc.log 2>&1 || exit 1
f=$(find /tmp/pmc8 -name "*counter_collection.csv" | head -1)
python3 tools/pmc_summary.py "$f" > $O/pmc_sf_b8_serial.txt || exit 1
head -60 $O/pmc_sf_b8_serial.txt
