#!/usr/bin/env python3
"""Overlap of communication / copies with compute in a rocprofv3 trace (--kernel-trace --memory-copy-trace
--output-format csv): for every RCCL kernel and every host<->device copy, the share of its duration during
which at least one compute kernel (anything else) was executing on the device.

    python3 tools/overlap_report.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv> [--last-ms 400]
"""
import argparse
import csv
import glob
import os
import sys


def load(path):
    return list(csv.DictReader(open(path))) if path else []


def merge(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(s, e, merged):
    c = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        c += min(b, e) - max(a, s)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-ms", type=float, default=0.0,
                    help="only the final window of this length before the last kernel ends (steady-state steps; "
                         "0 = everything, engine build and tuning included)")
    ap.add_argument("--dump", default="", help="write the window's kernels and copies to this CSV")
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    kern = load(kt[0] if kt else None)
    copies = load(mt[0] if mt else None)
    if not kern:
        print("no kernel trace")
        return 1
    t_end = max(int(r["End_Timestamp"]) for r in kern)
    t0 = t_end - int(a.last_ms * 1e6) if a.last_ms > 0 else min(int(r["Start_Timestamp"]) for r in kern)
    comm, compute = [], []
    for r in kern:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0:
            continue
        name = r["Kernel_Name"]
        (comm if ("nccl" in name.lower() or "rccl" in name.lower()) else compute).append((s, e, name))
    cm = merge([(s, e) for s, e, _ in compute])
    print(f"compute kernels: {len(compute)}, busy {sum(b - a for a, b in cm) / 1e6:.2f} ms")
    def report(tag, items):
        if not items:
            print(f"{tag}: none")
            return
        tot = sum(e - s for s, e, _ in items)
        ov = sum(covered(s, e, cm) for s, e, _ in items)
        print(f"{tag}: {len(items)} ops, {tot / 1e6:.3f} ms total, {ov / max(tot, 1) * 100:.1f}% of it concurrent "
              f"with compute kernels")
    report("RCCL kernels", comm)
    h2d = []
    for r in copies:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0:
            continue
        d = r.get("Direction", "")
        h2d.append((s, e, d))
    for d in sorted(set(x[2] for x in h2d)):
        report(f"copies {d}", [x for x in h2d if x[2] == d])
    if a.dump:
        # compact window dump (start/end relative to the window, ns) for offline timeline analysis
        with open(a.dump, "w") as f:
            f.write("kind,start_ns,end_ns,queue,name\n")
            for r in kern:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                if e >= t0:
                    f.write(f"k,{s - t0},{e - t0},{r.get('Queue_Id', '')},{r['Kernel_Name'][:60].replace(',', ';')}\n")
            for r in copies:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                if e >= t0:
                    f.write(f"c,{s - t0},{e - t0},,{r.get('Direction', '')}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
