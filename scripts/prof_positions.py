#!/usr/bin/env python3
"""Per-position kernel times of the timed bench steps (rocprofv3 kernel trace): the forward's launch sequence is the
same every step, so position i of every step is the same layer.  Prints, per position, the kernel, its grid, the
median / min / max duration over the steps and the gap to the previous kernel's end -- which launches are slow in
context (cold operands, clock, the previous kernel's tail), not only per kernel family.

Usage: prof_positions.py <kernel_trace.csv> [skip] [--top N] [--name SUBSTR]"""
import csv
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path, skip = args[0], int(args[1]) if len(args) > 1 else 3
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 0
    name = sys.argv[sys.argv.index("--name") + 1] if "--name" in sys.argv else None
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "tlc_scale_input" in r["Kernel_Name"]]
    blends = [i for i, r in enumerate(rows) if "tlc_blend" in r["Kernel_Name"]]
    steps = []
    for s in starts[skip:]:
        e = next(b for b in blends if b > s)
        steps.append(rows[s:e + 1])
    n = min(len(s) for s in steps)
    if any(len(s) != n for s in steps):
        print(f"# warning: steps have different dispatch counts {sorted(set(len(s) for s in steps))}")
    out = []
    for i in range(n):
        d = [(int(s[i]["End_Timestamp"]) - int(s[i]["Start_Timestamp"])) / 1e3 for s in steps]
        g = [(int(s[i]["Start_Timestamp"]) - int(s[i - 1]["End_Timestamp"])) / 1e3 for s in steps] if i else [0.0]
        r = steps[0][i]
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        out.append((i, short(r["Kernel_Name"]), r["Kernel_Name"], wg, statistics.median(d), min(d), max(d),
                    statistics.median(g)))
    tot = sum(o[4] for o in out)
    print(f"steps={len(steps)} positions={n} sum of medians={tot / 1e3:.3f} ms  gaps={sum(o[7] for o in out) / 1e3:.3f} ms")
    sel = [o for o in out if name is None or name in o[2]]
    if top:
        sel = sorted(sel, key=lambda o: -(o[4] - o[5]))[:top]
    for i, sn, full, wg, med, mn, mx, gap in sel:
        print(f"{i:4d} {med:8.1f} us  min {mn:7.1f} max {mx:7.1f} gap {gap:5.1f}  wg {wg:5d}  {sn[:40]}  {full[:110]}")


if __name__ == "__main__":
    main()
