#!/usr/bin/env python3
"""Per-step kernel breakdown of the timed bench region: dispatches between the start of the
(skip+1)-th tlc_scale_input and the end of the last tlc_blend, divided by the step count."""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main(path, skip):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "tlc_scale_input" in r["Kernel_Name"]]
    blends = [i for i, r in enumerate(rows) if "tlc_blend" in r["Kernel_Name"]]
    a, b = starts[skip], blends[-1]
    win = rows[a:b + 1]
    nsteps = len(starts) - skip
    wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e6
    by = defaultdict(lambda: [0, 0.0])
    tot = 0.0
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = short(r["Kernel_Name"])
        by[n][0] += 1
        by[n][1] += d
        tot += d
    print(f"steps={nsteps} wall/step={wall/nsteps:.3f} ms  kernel-sum/step={tot/1e3/nsteps:.3f} ms  "
          f"dispatches/step={len(win)/nsteps:.0f}")
    for n, (c, d) in sorted(by.items(), key=lambda x: -x[1][1]):
        print(f"{d/1e3/nsteps:8.3f} ms/step {100*d/tot:5.1f}%  calls/step {c/nsteps:6.1f}  avg {d/c:8.1f} us  {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
