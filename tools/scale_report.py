#!/usr/bin/env python3
"""Scaling-curve report: run ``bench.py --gpus N`` for N in {1, 2, 4, 8} (capped at the
visible GPU count unless ``--force``), one fresh job per N, and tabulate whole-job FPS, ms per step, ms per
frame per GPU, the all-gather time and the throughput scaling efficiency relative to N = 1.

    python tools/scale_report.py --steps 20 --warmup 5 --out profiles/scale.md
    SA_DIST_BACKEND=gloo python tools/scale_report.py --device cpu ...   # plumbing rehearsal on the CPU

Each N runs as its own process tree (bench.py self-launches its ranks), so a failing N is reported and the
sweep continues.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def run_one(n: int, bench_args: list[str], timeout: int) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    t0 = time.time()
    try:
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--no-latency", *bench_args],
                           env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"n": n, "error": f"timeout after {timeout}s"}
    wall = time.time() - t0
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"n": n, "error": f"rc={r.returncode}: {r.stderr.strip()[-400:]}"}
    rec = json.loads(lines[-1])
    rec["wall_s"] = round(wall, 1)
    return rec


def table(rows: list[dict]) -> str:
    base = next((r for r in rows if r.get("n_gpus") == 1 and "error" not in r), None)
    out = ["| GPUs | whole-job FPS | ms / step | ms / frame / GPU | all-gather ms | scaling eff. | config |",
           "|---|---|---|---|---|---|---|"]
    for r in rows:
        if "error" in r:
            out.append(f"| {r['n']} | — | — | — | — | — | failed: {r['error'][:80]} |")
            continue
        eff = r["value"] / (base["value"] * r["n_gpus"]) if base else None
        out.append(f"| {r['n_gpus']} | {r['value']:.1f} | {r['ms_per_step']:.2f} | {r['ms_per_frame_per_gpu']:.3f} | "
                   f"{r.get('allgather_ms') if r.get('allgather_ms') is not None else '—'} | "
                   f"{'%.3f' % eff if eff else '—'} | {r['config']['model']} b{r['config']['per_gpu_batch']}/GPU "
                   f"{r['config']['resolution']} {r['config']['parallelism']} |")
    return "\n".join(out)


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--sizes", default="1,2,4,8")
    p.add_argument("--force", action="store_true", help="do not cap N at the visible GPU count")
    p.add_argument("--timeout", type=int, default=900)
    p.add_argument("--out", default=None, help="write the markdown table (and a .json next to it)")
    args, bench_args = p.parse_known_args(argv)
    sizes = [int(s) for s in args.sizes.split(",")]
    if not args.force and "cpu" not in bench_args:
        import torch
        ndev = torch.cuda.device_count()
        capped = [n for n in sizes if n <= max(ndev, 1)]
        if capped != sizes:
            print(f"[scale] {ndev} GPU(s) visible: running N in {capped}", file=sys.stderr)
        sizes = capped
    rows = []
    for n in sizes:
        rec = run_one(n, bench_args, args.timeout)
        rows.append(rec)
        print(f"[scale] N={n}: " + (rec.get("error") or f"{rec['value']} FPS, {rec['ms_per_step']} ms/step"),
              file=sys.stderr, flush=True)
    md = table(rows)
    print(md)
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(md + "\n")
        Path(args.out).with_suffix(".json").write_text(json.dumps(rows, indent=1) + "\n")
    return 0 if all("error" not in r for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
