#!/usr/bin/env python3
"""Per-frame / per-iteration timeline of a replayed frame graph from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -- python3 tools/run_engine.py --frames 4 ...
    python3 tools/timeline.py gpurun_out/tl [--frame-marker preprocess] [--iter-marker motion_encoder]

For the last complete frame (frames start at the first `--frame-marker` kernel after a gap) it prints:
  * frame span, device-busy time (union of kernel intervals), idle time and the number of idle gaps;
  * per iteration (delimited by `--iter-marker` kernels): span, busy, idle, kernel count;
  * the critical chain, walked backwards from the frame's last kernel: each link is the kernel whose end is
    the latest end at or before the current kernel's start (the dependency that released it, assuming a kernel
    starts as soon as its last input is ready), with the launch gap of every link;
  * per-kernel-name totals on the critical chain vs off it.
Kernel durations of concurrent kernels overlap, so per-kernel sums exceed the span; the busy union does not.
"""
import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True) if os.path.isdir(d) else [d]
    if not files:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
            gy = int(r.get("Grid_Size_Y", 1) or 1)
            gz = int(r.get("Grid_Size_Z", 1) or 1)
            wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
            wy = int(r.get("Workgroup_Size_Y", 1) or 1)
            wz = int(r.get("Workgroup_Size_Z", 1) or 1)
            wgs = max(1, (gx // max(wx, 1)) * (gy // max(wy, 1)) * (gz // max(wz, 1)))
            q = int(r.get("Queue_Id", -1) or -1)
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), wgs, q))
    rows.sort()
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n)
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)(\w+)", n)
    if m:
        ln = int(m.group(1))
        n = m.group(2)[:ln]
    n = n.replace("conv_igemm_kernel", "igemm").replace(", false>", ">")
    return n[:60]


def union(iv):
    tot, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in sorted(iv):
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            tot += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def frames(rows, marker, min_gap_ns):
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    # a frame begins at a marker kernel that is not within min_gap of the previous marker (RAFT preprocesses L and R)
    fs = []
    for i in starts:
        if not fs or rows[i][0] - rows[fs[-1]][0] > min_gap_ns:
            fs.append(i)
    return fs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frame-marker", default="preprocess")
    ap.add_argument("--iter-marker", default="")
    ap.add_argument("--frame", type=int, default=-2, help="which frame (python index over complete frames)")
    ap.add_argument("--chain", type=int, default=60, help="critical-chain links to print (from the end)")
    ap.add_argument("--list", type=int, default=0, help="print the first N kernels of the frame in start order")
    ap.add_argument("--kernel-stats", type=int, default=0,
                    help="per-kernel dispatch counts and device time of THIS frame replay only (top N), so no tuning "
                         "pass or eager launch is averaged into 'per frame'")
    a = ap.parse_args()
    rows = load(a.trace)
    fs = frames(rows, a.frame_marker, 200_000)
    if len(fs) < 2:
        sys.exit(f"found {len(fs)} frame markers")
    bounds = list(zip(fs[:-1], fs[1:]))
    lo, hi = bounds[a.frame]
    fr = rows[lo:hi]
    # drop the tail of foreign kernels after the frame's last kernel (next frame's host copies etc.)
    t0 = fr[0][0]
    t1 = max(r[1] for r in fr)
    busy, gaps = union([(r[0], r[1]) for r in fr])
    span = t1 - t0
    print(f"frame {a.frame}: {len(fr)} kernels, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us "
          f"({100 * busy / span:.1f} %), idle {(span - busy) / 1e3:.1f} us in {len(gaps)} gaps "
          f"(>5us: {sum(1 for g in gaps if g > 5000)}, sum {sum(g for g in gaps if g > 5000) / 1e3:.1f} us)")
    if a.kernel_stats:
        agg = {}
        for s_, e_, n, w, q in fr:
            k = short(n)
            c, t = agg.get(k, (0, 0))
            agg[k] = (c + 1, t + (e_ - s_))
        tot = sum(t for _, t in agg.values())
        print(f"\nper-kernel device time in this frame replay ({len(fr)} dispatches, {tot / 1e3:.1f} us summed over "
              f"queues; concurrent kernels overlap, so the sum exceeds the span)")
        print(f"  {'kernel':62s} {'n':>4s} {'us':>9s} {'avg us':>8s} {'%':>6s}")
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.kernel_stats]:
            print(f"  {k:62s} {c:4d} {t / 1e3:9.1f} {t / c / 1e3:8.2f} {100 * t / tot:6.2f}")
    if a.list:
        for s, e, n, w, q in fr[:a.list]:
            print(f"  +{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  wg {w:6d}  q{q}  {n}")

    if a.iter_marker:
        its = [i for i, r in enumerate(fr) if a.iter_marker in r[2]]
        print(f"\n{len(its)} iterations (marker '{a.iter_marker}')")
        spans = []
        for k, (i, j) in enumerate(zip(its, its[1:] + [len(fr)])):
            seg = fr[i:j]
            s0 = seg[0][0]
            s1 = fr[j][0] if j < len(fr) else max(r[1] for r in seg)
            b, g = union([(r[0], min(r[1], s1)) for r in seg])
            spans.append(s1 - s0)
            if k < 3 or k >= len(its) - 2 or k == len(its) // 2:
                print(f"  it {k:2d}: span {(s1 - s0) / 1e3:7.1f} us  busy {b / 1e3:7.1f}  idle {(s1 - s0 - b) / 1e3:6.1f} "
                      f"in {len(g)} gaps  kernels {len(seg)}")
        if spans:
            ss = sorted(spans[1:-1]) or spans
            print(f"  median iteration span {ss[len(ss) // 2] / 1e3:.1f} us")

    # critical chain: from the last-ending kernel, repeatedly take the latest-ending kernel that ended at or before
    # this one's start (+1 us slack for timestamp skew)
    idx = max(range(len(fr)), key=lambda i: fr[i][1])
    chain = [idx]
    by_end = sorted(range(len(fr)), key=lambda i: fr[i][1])
    ends = [fr[i][1] for i in by_end]
    import bisect
    while True:
        s = fr[chain[-1]][0]
        p = bisect.bisect_right(ends, s + 1000) - 1
        # a predecessor started before this kernel did (the slack must not admit a concurrent branch that began
        # after it and happened to end within the slack)
        while p >= 0 and (by_end[p] == chain[-1] or fr[by_end[p]][0] >= s):
            p -= 1
        if p < 0:
            break
        chain.append(by_end[p])
        if fr[by_end[p]][0] <= t0:
            break
    chain.reverse()
    tot_k = sum(fr[i][1] - fr[i][0] for i in chain)
    tot_gap = sum(max(0, fr[j][0] - fr[i][1]) for i, j in zip(chain, chain[1:]))
    print(f"\ncritical chain: {len(chain)} kernels, {tot_k / 1e3:.1f} us in kernels + {tot_gap / 1e3:.1f} us of "
          f"launch gaps = {(tot_k + tot_gap) / 1e3:.1f} us (frame span {span / 1e3:.1f})")
    # links by hardware queue: a link between kernels of different queues is a graph edge the executor turned into
    # a barrier packet (rocprofv3 Queue_Id; -1 when the trace has none)
    same = [max(0, fr[j][0] - fr[i][1]) for i, j in zip(chain, chain[1:]) if fr[i][4] == fr[j][4]]
    cross = [max(0, fr[j][0] - fr[i][1]) for i, j in zip(chain, chain[1:]) if fr[i][4] != fr[j][4]]
    print(f"  links: {len(same)} same-queue ({sum(same) / 1e3:.1f} us of gaps), {len(cross)} cross-queue "
          f"({sum(cross) / 1e3:.1f} us of gaps, {sum(cross) / max(1, len(cross)) / 1e3:.1f} us each)")
    per = defaultdict(lambda: [0, 0, 0])
    for i, j in zip([None] + chain[:-1], chain):
        s, e, n, w, _ = fr[j]
        g = 0 if i is None else max(0, s - fr[i][1])
        per[n][0] += 1
        per[n][1] += e - s
        per[n][2] += g
    print(f"  {'kernel':60s} {'n':>4s} {'kern us':>9s} {'gap us':>8s}")
    for n, (c, k, g) in sorted(per.items(), key=lambda x: -x[1][1] - x[1][2]):
        print(f"  {n:60s} {c:4d} {k / 1e3:9.1f} {g / 1e3:8.1f}")
    print(f"\n  last {a.chain} links:")
    for i, j in list(zip([None] + chain[:-1], chain))[-a.chain:]:
        s, e, n, w, q = fr[j]
        g = 0 if i is None else s - fr[i][1]
        print(f"  +{(s - t0) / 1e3:9.1f}  gap {g / 1e3:6.1f}  dur {(e - s) / 1e3:7.1f}  wg {w:6d}  q{q:<2d} {n}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
