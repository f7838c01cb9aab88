#!/usr/bin/env python3
"""Per-step GEMM time by kernel instance (template args) and grid size, from a rocprofv3 kernel trace."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "tlc_scale_input" in r["Kernel_Name"]]
blends = [i for i, r in enumerate(rows) if "tlc_blend" in r["Kernel_Name"]]
skip = 2
win = rows[starts[skip]:blends[-1] + 1]
n = len(starts) - skip
by = defaultdict(list)
for r in win:
    k = r["Kernel_Name"]
    if "gemm" not in k and "conv_halo" not in k:
        continue
    m = re.search(r"(gemm8?_kernel|conv_halo_kernel)I(.*?)Ev14fd_", k)
    targs = (m.group(1) + " " + m.group(2)) if m else k[:60]
    targs = targs.replace("DF16b", "bf16").replace("DF16_", "f16")
    by[(targs, r["Grid_Size_X"], r["Workgroup_Size_X"])].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0
for k, v in sorted(by.items(), key=lambda x: -sum(x[1])):
    tot += sum(v)
    print(f"{sum(v) / n / 1e3:7.3f} ms/step  n/step {len(v) / n:5.1f} avg {sum(v) / len(v):7.1f} min {min(v):7.1f}  "
          f"wg {int(k[1]) // int(k[2]):6d}  {k[0]}")
print(f"total {tot / n / 1e3:.3f} ms/step")
