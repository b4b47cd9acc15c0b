#!/usr/bin/env python3
"""Regression gate: compare a fresh bench.py JSON line against the previous round's driver record.

    python3 tools/bench_regress.py gpurun_out/r5b/bench.log [--baseline BENCH_r04.json] [--tol 0.03]

The baseline defaults to the newest BENCH_r*.json at the repository root (the driver's own run of bench.py on a fresh
box at the end of a round).  Compared: the headline throughput (higher is better) and, per preset of the batch-1
block, the caller-buffer latency and the network-only device time (lower is better).  Exits 1 when any of them is
worse than the baseline by more than --tol (default 3 %), printing every row either way.  Cross-box spread on this
pool is a few percent (profiles/round4_notes.md), so a failing row is re-measured before it is believed -- but a
change that moves a preset by more than that spread is what VERDICT r4 weak #2 asked to catch (CREStereo +5.7 %
across a round, unnoticed).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys


def last_json_line(path: str) -> dict:
    with open(path) as f:
        text = f.read()
    if path.endswith(".json") and text.lstrip().startswith("{") and '"parsed"' in text:
        rec = json.loads(text)  # a driver BENCH_rNN.json: the bench line is in run.stdout_tail
        tail = rec.get("run", {}).get("stdout_tail", "") or rec.get("tail", "")
        text = tail
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise ValueError(f"{path}: no bench JSON line found")


def newest_baseline(root: str) -> str | None:
    files = glob.glob(os.path.join(root, "BENCH_r*.json"))
    files.sort(key=lambda f: int(re.search(r"BENCH_r(\d+)", f).group(1)))
    return files[-1] if files else None


def network_ms(stages: dict) -> float | None:
    """Device time of the network: the sum of the stage marks other than the input read, the rectification and the
    reprojection (round 5 moved the input copy into the frame graph as its own "input" stage)."""
    if not stages:
        return None
    return round(sum(v for k, v in stages.items() if k not in ("input", "reproject", "rectify")), 3)


def compare(new: dict, base: dict, tol: float):
    rows = []
    rows.append(("throughput (frames/s)", base["value"], new["value"], True))
    nb, bb = new.get("latency_b1") or {}, base.get("latency_b1") or {}
    for preset in bb:
        if preset not in nb:
            continue
        rows.append((f"{preset} latency ms", bb[preset]["latency_ms_mean"], nb[preset]["latency_ms_mean"], False))
        a, b = network_ms(bb[preset].get("device_stages_ms")), network_ms(nb[preset].get("device_stages_ms"))
        if a and b:
            rows.append((f"{preset} network ms", a, b, False))
    out, bad = [], 0
    for name, old, cur, higher in rows:
        rel = (cur - old) / old if old else 0.0
        worse = -rel if higher else rel
        flag = worse > tol
        bad += flag
        out.append(f"{'REGRESSION' if flag else 'ok':10s} {name:40s} {old:10.3f} -> {cur:10.3f}  ({rel * 100:+6.2f} %)")
    return out, bad


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("fresh", help="bench.py output (log whose last JSON line is the record) or a BENCH_rNN.json")
    ap.add_argument("--baseline", default=None, help="baseline record (default: newest BENCH_r*.json at the repo root)")
    ap.add_argument("--tol", type=float, default=0.03)
    a = ap.parse_args(argv)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base_path = a.baseline or newest_baseline(root)
    if not base_path:
        print("no baseline BENCH_r*.json found", file=sys.stderr)
        return 2
    rows, bad = compare(last_json_line(a.fresh), last_json_line(base_path), a.tol)
    print(f"baseline {os.path.basename(base_path)}, tolerance {a.tol * 100:.1f} %")
    print("\n".join(rows))
    print(f"{bad} regression(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
