#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per kernel (and grid) total time, calls, and per-step share."""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"_Z\d+(\w+?)I", name)
    base = m.group(1) if m else name[:40]
    if "gemm8_kernel" in name:
        t = re.search(r"gemm8_kernelI(DF16b|DF16_)Li(\d+)ELi(\d+)ELb(\d)ELb(\d)E", name)
        if t:
            dt = "bf16" if t.group(1) == "DF16b" else "f16"
            kind = "conv" if t.group(4) == "1" else ("geglu" if t.group(5) == "1" else "gemm")
            return f"gemm8[{kind},{dt},256x{t.group(2)}]"
    if "gemm_kernel" in name:
        t = re.search(r"gemm_kernelI(DF16b|DF16_)Li(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELb(\d)E(\w+?)Ev", name)
        if t:
            dt = "bf16" if t.group(1) == "DF16b" else "f16"
            kind = "conv" if t.group(6) == "1" else ("geglu" if t.group(7) == "1" else "gemm")
            return f"gemm[{kind},{dt},{t.group(2)}x{t.group(3)}]"
    return base


def main(path, per=1):
    rows = list(csv.DictReader(open(path)))
    by = defaultdict(lambda: [0, 0.0])
    byg = defaultdict(lambda: [0, 0.0])
    tot = 0.0
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
        n = short(r["Kernel_Name"])
        g = (r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))
        by[n][0] += 1
        by[n][1] += d
        byg[(n, g)][0] += 1
        byg[(n, g)][1] += d
        tot += d
    print(f"total kernel time {tot/1e3:.2f} ms over {len(rows)} dispatches; per unit (/{per}) {tot/1e3/per:.2f} ms")
    for n, (c, d) in sorted(by.items(), key=lambda x: -x[1][1])[:25]:
        print(f"{d/1e3/per:9.3f} ms/unit {100*d/tot:5.1f}%  calls/unit {c/per:7.1f}  avg {d/c:8.1f} us  {n}")
    print("-- top (kernel, grid)")
    for (n, g), (c, d) in sorted(byg.items(), key=lambda x: -x[1][1])[:30]:
        print(f"{d/1e3/per:9.3f} ms/unit {100*d/tot:5.1f}%  calls/unit {c/per:6.1f}  avg {d/c:8.1f} us  {n} grid={g}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1)
