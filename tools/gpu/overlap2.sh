# Overlap evidence at HEAD defaults (batch 8: 2 engine streams): bench.py DP step at world 1 with the
# collective forced on (H2D prefetch vs frame graph), and the native RCCL runner (ncclAllGather on its comm
# stream vs the next frame graph).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export SA_PLAN_DIR=/tmp/sa_plans
SA_DP_GATHER_WORLD1=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-latency > /dev/null 2>&1 || exit 1
rm -rf gpurun_out/ovp
SA_DP_GATHER_WORLD1=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d gpurun_out/ovp -o run -- python3 bench.py --steps 6 --warmup 2 --no-latency > gpurun_out/ovp.log 2>&1 || exit 1
echo "== bench.py DP step, world 1, gather forced (HEAD defaults)"
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ovp.log
python3 tools/overlap_report.py gpurun_out/ovp --last-ms 380
rm -rf gpurun_out/ovn
SA_DP_GATHER_WORLD1=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d gpurun_out/ovn -o run -- stereoalgorithms_amd/bin/stereo_bench_dp --nproc 0 --batch 8 --steps 6 --warmup 2 \
  > gpurun_out/ovn.log 2>&1 || exit 1
echo "== native RCCL runner, world 1, gather forced"
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ovn.log
python3 tools/overlap_report.py gpurun_out/ovn --last-ms 380
f=$(find gpurun_out/ovn -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
c = collections.Counter(r["Kernel_Name"][:60] for r in csv.DictReader(open(sys.argv[1])) if "nccl" in r["Kernel_Name"].lower() or "rccl" in r["Kernel_Name"].lower())
print("RCCL kernel names:", dict(c))
PY
rm -rf gpurun_out/ovp gpurun_out/ovn
