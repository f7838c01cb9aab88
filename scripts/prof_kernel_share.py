#!/usr/bin/env python3
"""Per-forward kernel time by (kernel instance, grid) over the denoise loop of a rocprofv3 kernel trace: the window
from the third fd_tlc_scale_input launch to the last tlc_blend, normalised by the scale-input launches in it (one per
UNet forward, i.e. per tile batch in the tiled C3 / C4 loops); with [last] > 0 the window starts at the last-th
scale-input launch from the end instead (the final denoise loop only, when the trace also holds warm-up calls and
their VAE work).  Prints the top instances and a per-family total.

    python scripts/prof_kernel_share.py <kernel_trace.csv> [top] [last]
"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "tlc_scale_input" in r["Kernel_Name"]]
blends = [i for i, r in enumerate(rows) if "tlc_blend" in r["Kernel_Name"]]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
first = len(starts) - last if last > 0 else 2
win = rows[starts[first]:blends[-1] + 1]
n = len(starts) - first
by, fam = defaultdict(list), defaultdict(float)
for r in win:
    k = r["Kernel_Name"]
    m = re.search(r"(\w+?_kernel)I(.*?)Ev", k)
    name = (m.group(1) + " " + m.group(2)[:70]) if m else re.sub(r"\(.*", "", k)[:80]
    name = name.replace("DF16b", "bf16").replace("DF16_", "f16")
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by[(name, r["Grid_Size_X"], r["Workgroup_Size_X"])].append(us)
    fam[m.group(1) if m else name.split()[0]] += us
span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
print(f"{n} forwards in the window, {span / n / 1e3:.3f} ms wall per forward, "
      f"{sum(fam.values()) / n / 1e3:.3f} ms kernel sum per forward")
for k, v in sorted(by.items(), key=lambda x: -sum(x[1]))[:top]:
    print(f"{sum(v) / n / 1e3:7.3f} ms/fwd  n/fwd {len(v) / n:5.1f} avg {sum(v) / len(v):8.1f} us  "
          f"wg {int(k[1]) // max(1, int(k[2])):7d}  {k[0]}")
print("-- by family")
for k, v in sorted(fam.items(), key=lambda x: -x[1]):
    print(f"{v / n / 1e3:7.3f} ms/fwd  {k}")
