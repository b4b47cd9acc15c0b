#!/usr/bin/env python3
"""Per-kernel register / spill / LDS / occupancy summary of one HIP source for gfx950.

    python tools/res_usage.py csrc/kernels/conv2d.hip [name-filter-regex]
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    filt = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Icsrc/include", "-c", src,
           "-o", "/tmp/_res_usage.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.+?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    for r in rows:
        if filt and not filt.search(r["name"]):
            continue
        print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a  spill s{r.get('SGPRs Spill', '?'):>4} "
              f"v{r.get('VGPRs Spill', '?'):>4}  lds {r.get('LDS Size [bytes/block]', '?'):>6}  "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}  {r['name']}")


if __name__ == "__main__":
    main()
