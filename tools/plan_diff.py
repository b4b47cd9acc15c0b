#!/usr/bin/env python3
"""Compare two tuned-plan files (csrc/runtime/runtime.cpp format): per conv key the tactic / split and the timed us,
keys only in one file listed, and the summed tuned time of the keys both files hold.

    python3 tools/plan_diff.py old.plan new.plan
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereoalgorithms_amd.utils.plan import read_plan  # noqa: E402


def main():
    a_build, a = read_plan(sys.argv[1])
    b_build, b = read_plan(sys.argv[2])
    am = {e.key.replace("|b", ""): e for e in a}
    bm = {e.key.replace("|b", ""): e for e in b}
    print(f"# {sys.argv[1]} (build {a_build}, {len(a)} keys) vs {sys.argv[2]} (build {b_build}, {len(b)} keys)")
    both = sorted(set(am) & set(bm))
    ta = tb = 0.0
    for k in both:
        ea, eb = am[k], bm[k]
        ta += ea.us
        tb += eb.us
        mark = "" if (ea.cfg, ea.splitk) == (eb.cfg, eb.splitk) else "  *"
        print(f"{k[:96]:96s} cfg {ea.cfg:2d}/{ea.splitk:2d} {ea.us:8.1f} -> cfg {eb.cfg:2d}/{eb.splitk:2d} {eb.us:8.1f}{mark}")
    for k in sorted(set(am) - set(bm)):
        print(f"only old: {k[:100]}")
    for k in sorted(set(bm) - set(am)):
        print(f"only new: {k[:100]}")
    print(f"sum of tuned times over {len(both)} shared keys: {ta:.1f} -> {tb:.1f} us")


if __name__ == "__main__":
    main()
