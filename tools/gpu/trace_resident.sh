#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ovr_${MODE:-resident}; mkdir -p $O
rm -rf /tmp/ovr_${MODE:-resident}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/ovr_${MODE:-resident} -o run -- python3 tools/exp/dp_h2d_variants.py ${MODE:-resident} > $O/trace.log 2>&1 || exit 1
grep -E "ms/step" $O/trace.log
python3 tools/overlap_report.py /tmp/ovr_${MODE:-resident} --last-ms 600 --dump $O/window.csv
