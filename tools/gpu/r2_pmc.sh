# MFMA busy fraction (at the clock the chip held) of the headline's hot convs and the new encoder kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
pass() {  # name shapes cfgs match
  rm -rf gpurun_out/pmc_$1
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_$1 -o run -- python3 tools/conv_bench.py --iters 5 --shapes $2 --cfgs $3 > gpurun_out/pmc_$1.log 2>&1 || return 1
  f=$(find gpurun_out/pmc_$1 -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py "$f" --match $4 > gpurun_out/pmc_$1.txt
  rm -rf gpurun_out/pmc_$1
}
pass gru zr8,q8,fh8 4,15 conv_igemm && pass d64 fr8 23 conv3x3 && pass d96 l2b8,l2s8 24 conv3x3 && pass stem stem8 22 conv7x7
for n in gru d64 d96 stem; do echo "== $n"; grep -v amdgpu gpurun_out/pmc_$n.log | grep "TFLOP"; cat gpurun_out/pmc_$n.txt; done > gpurun_out/pmc_r02.txt; cat gpurun_out/pmc_r02.txt | grep -E "==|TFLOP|held clock|  grid"
