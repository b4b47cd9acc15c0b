#!/bin/bash
# Kernel-level times of the workgroup split-K tactics (37 / 38) against the deep-ring tile (16) on the coarse GRU
# shapes: the split tests, then rocprofv3 kernel stats of tools/conv_bench.py, one run per tactic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sxp
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "workgroup_splitk or gru_zrq_split" > gpurun_out/sxp/pytest.log 2>&1 || { tail -30 gpurun_out/sxp/pytest.log; exit 1; }
tail -1 gpurun_out/sxp/pytest.log
for c in 16 37 38; do
  rm -rf /tmp/sxp_$c
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sxp_$c -o run -- python3 tools/conv_bench.py \
      --shapes ${SHAPES:-zr32,q32,zr8l,q8l} --cfgs $c --splits 1 --iters 50 > gpurun_out/sxp/bench_$c.log 2>&1 || exit 1
  f=$(find /tmp/sxp_$c -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/sxp/stats_$c.csv
  grep cfg gpurun_out/sxp/bench_$c.log | grep -v W2026
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'conv' in r['Name']:
        print('   ', r['Name'].split('(anonymous namespace)::')[-1][:60], r['Calls'], '%.2f us' % (float(r['AverageNs']) / 1e3))
PY
done
