#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv: per (kernel, grid) the median of each counter over
dispatches, plus derived MFMA busy fraction when SQ_VALU_MFMA_BUSY_CYCLES and SQ_BUSY_CYCLES are present.

    python3 tools/pmc_summary.py gpurun_out/pmc/run_counter_collection.csv [--match conv_igemm]
"""
import argparse
import csv
import re
import statistics
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="", help="regex on the kernel name")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    if not rows:
        print("no rows")
        return 1
    kcol = "Kernel_Name" if "Kernel_Name" in rows[0] else "Kernel-Name"
    data = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [per-dispatch values]
    disp = defaultdict(lambda: defaultdict(float))  # (kernel, grid, dispatch) -> counter -> summed value
    for r in rows:
        k = r[kcol]
        if a.match and not re.search(a.match, k):
            continue
        g = r.get("Grid_Size") or r.get("Grid-Size") or ""
        d = r.get("Dispatch_Id") or r.get("Dispatch-Id") or ""
        disp[(k, g, d)][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, g, d), cs in disp.items():
        for c, v in cs.items():
            data[(k, g)][c].append(v)
    for (k, g), cs in sorted(data.items()):
        print(f"{k[:110]}  grid {g}")
        med = {c: statistics.median(v) for c, v in cs.items()}
        for c, v in sorted(med.items()):
            print(f"  {c:32s} {v:.4g}  (n={len(cs[c])})")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "SQ_BUSY_CYCLES" in med and med["SQ_BUSY_CYCLES"] > 0:
            # SQ_BUSY_CYCLES counts per SE (32 on MI355X); MFMA busy is per SIMD (1024 SIMDs)
            print(f"  -> MFMA busy / (SQ_BUSY_CYCLES x 1024 / 32): "
                  f"{med['SQ_VALU_MFMA_BUSY_CYCLES'] / (med['SQ_BUSY_CYCLES'] * 1024 / 32):.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med and med.get("GRBM_GUI_ACTIVE", 0) > 0:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs: /8 = the dispatch's cycles at the clock it actually held
            # (MI355X_MICROARCH.md 'DVFS give-back'); MFMA busy cycles are summed over the 1024 SIMDs
            print(f"  -> MFMA busy fraction at the held clock, busy / (GRBM_GUI_ACTIVE / 8 x 1024): "
                  f"{med['SQ_VALU_MFMA_BUSY_CYCLES'] / (med['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
