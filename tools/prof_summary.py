#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database: per-kernel totals and per-(kernel, grid) breakdown.

    python3 tools/prof_summary.py gpurun_out/prof/run_results.db [--frames N] [--top 40]
"""
import argparse
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--frames", type=int, default=1, help="divide totals by this (per-frame numbers)")
    p.add_argument("--top", type=int, default=40)
    p.add_argument("--by-grid", action="store_true")
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    tot = c.execute("select sum(duration) from kernels").fetchone()[0] or 0
    print(f"total kernel time {tot / 1e6:.3f} ms ({tot / 1e6 / a.frames:.3f} ms per frame), "
          f"{c.execute('select count(*) from kernels').fetchone()[0] / a.frames:.0f} dispatches per frame")
    # template arguments of conv_igemm_kernel<BM, BN, WM, WN, MODE> from the mangled symbol
    import re
    sym = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}

    def label(name, kid):
        m = re.search(r"ILi(\d+)ELi(\d+)ELi\d+ELi\d+ELi(\d)E", sym.get(kid, ""))
        if name == "conv_igemm_kernel" and m:
            return f"conv<{m.group(1)}x{m.group(2)},{['k32', 'dma64', 'k64'][int(m.group(3))]}>"
        return name

    key = "name, kernel_id, grid_x, grid_y, grid_z, workgroup_x" if a.by_grid else "name, kernel_id"
    q = (f"select {key}, count(*), sum(duration), avg(duration) from kernels group by {key} "
         f"order by sum(duration) desc limit {a.top}")
    print(f"{'kernel':70s} {'grid':>18s} {'calls/fr':>8s} {'ms/fr':>9s} {'avg us':>9s} {'%':>6s}")
    for r in c.execute(q):
        name = label(r[0], r[1])[:70]
        if a.by_grid:
            grid = f"{r[2]}x{r[3]}x{r[4]}/{r[5]}"
            n, s, avg = r[6], r[7], r[8]
        else:
            grid, n, s, avg = "", r[2], r[3], r[4]
        print(f"{name:70s} {grid:>18s} {n / a.frames:8.1f} {s / 1e6 / a.frames:9.3f} {avg / 1e3:9.2f} "
              f"{100 * s / tot:6.2f}")

if __name__ == "__main__":
    main()
