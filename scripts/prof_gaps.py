#!/usr/bin/env python3
"""Launch-gap anatomy of graph-replayed denoise steps in a rocprofv3 kernel trace: per step, wall time vs
summed kernel time, the idle time between consecutive dispatches, and the largest gaps with their neighbours."""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main(path, skip=2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "tlc_scale_input" in r["Kernel_Name"]]
    blends = [i for i, r in enumerate(rows) if "tlc_blend" in r["Kernel_Name"]]
    a, b = starts[skip], blends[-1]
    win = rows[a:b + 1]
    nsteps = len(starts) - skip
    gaps = []
    busy = 0.0
    for i, r in enumerate(win):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += (e - s) / 1e3
        if i:
            gaps.append(((s - int(win[i - 1]["End_Timestamp"])) / 1e3, short(win[i - 1]["Kernel_Name"]),
                         short(r["Kernel_Name"])))
    wall = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
    gsum = sum(max(g[0], 0) for g in gaps)
    print(f"steps={nsteps} dispatches/step={len(win)/nsteps:.0f} wall/step={wall/nsteps/1e3:.3f} ms "
          f"kernel-sum/step={busy/nsteps/1e3:.3f} ms idle/step={gsum/nsteps/1e3:.3f} ms "
          f"mean gap={gsum/max(len(gaps),1):.2f} us")
    pos = sorted(g[0] for g in gaps)
    if pos:
        print("gap percentiles us: p10 %.2f p50 %.2f p90 %.2f p99 %.2f" % tuple(pos[int(q * (len(pos) - 1))] for q in (0.1, 0.5, 0.9, 0.99)))
    for g in sorted(gaps, reverse=True)[:15]:
        print(f"  {g[0]:8.2f} us  {g[1]} -> {g[2]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
