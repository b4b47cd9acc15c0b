# PMC passes (one counter group per run) over conv_bench shapes for a few tile configs.
#   SHAPES=zr8 CFGS=4,10 bash tools/gpu/pmc_conv.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${SHAPES:-zr8}
C=${CFGS:-4,10}
pass() {  # name counters...
  local n=$1; shift
  rm -rf gpurun_out/pmc_$n
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc "$@" -d gpurun_out/pmc_$n -o run -- python3 tools/conv_bench.py --iters 5 --shapes $S --cfgs $C > gpurun_out/pmc_$n.log 2>&1 || return 1
  f=$(find gpurun_out/pmc_$n -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py "$f" --match conv_igemm > gpurun_out/pmc_$n.txt
  rm -rf gpurun_out/pmc_$n
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE && \
pass b SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES && \
pass c TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_BUSY_CYCLES
cat gpurun_out/pmc_a.txt gpurun_out/pmc_b.txt gpurun_out/pmc_c.txt
