#!/bin/bash
# PMC passes (one counter group per run, --kernel-trace free) over a serialized engine frame, plans tuned beforehand
# in a separate unprofiled process so no tuning-pass launch is counted.
#   MODEL=raftstereo-sceneflow BATCH=8 MATCH="conv_igemm|motion_encoder|tapproj" bash tools/gpu/pmc_engine.sh tag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-pmce}
M=${MODEL:-raftstereo-sceneflow}
B=${BATCH:-8}
mkdir -p gpurun_out/$T
export SA_PLAN_CACHE=/tmp/sa_plan_pmc_$T.txt SA_RAFT_PARALLEL=0 SA_RAFT_PIPELINE=0
rm -f $SA_PLAN_CACHE
timeout -k 10 200 python3 tools/run_engine.py --model $M --batch $B --frames 1 > gpurun_out/$T/tune.log 2>&1 || exit 1
pass() {  # name counters...
  local n=$1; shift
  rm -rf /tmp/pmc_$T_$n
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc "$@" -d /tmp/pmc_${T}_$n -o run -- \
    python3 tools/run_engine.py --model $M --batch $B --frames 1 > gpurun_out/$T/pmc_$n.log 2>&1 || return 1
  f=$(find /tmp/pmc_${T}_$n -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py "$f" --match "${MATCH:-}" > gpurun_out/$T/pmc_$n.txt
  rm -rf /tmp/pmc_${T}_$n
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE && \
pass b SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES && \
cat gpurun_out/$T/pmc_a.txt gpurun_out/$T/pmc_b.txt
