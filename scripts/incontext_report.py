#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of scripts/incontext_probe.py into its phases (fd_postprocess_u8 markers around
each phase's replays) and compare the same launches in context (the forward graph) and in their family graphs.

For every (kernel, grid) key of the `proj` and `flash` family phases -- and per kernel family over all launches --
it reports, in each phase: launches, mean / median / min duration, and, with the clock sampler's samples
(<tag>_samples.npz from the same traced run), the mean shader clock over each launch's lifetime and the launch's
length in shader cycles (duration x clock).  The sampler kernel (clk_kernel) is in the trace, so sample i sits at
its Start_Timestamp + (realtime_i - realtime_0) * 10 ns.  With a PMC counter CSV of TCC_HIT_sum / TCC_MISS_sum (same
phases) it adds the L2 hit rate of those launches per phase.

    python scripts/incontext_report.py <kernel_trace.csv[.gz]> [--samples s.npz] [--pmc counter_collection.csv[.gz]]
"""
import bisect
import csv
import gzip
import json
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

PHASES = ["forward", "proj", "flash", "gemm"]


def rows_of(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        return list(csv.DictReader(f))


def grid(r):
    return int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)


def family(name):
    for key, fam in (("flash_attn_d64", "flash_d64"), ("gemm8_kernel", "gemm8"), ("gemm_kernel", "gemm4w"),
                     ("gemm256_kernel", "gemm256"), ("conv_halo", "conv_halo")):
        if key in name:
            return fam
    return "other"


def split(rows, key):
    rows = sorted(rows, key=lambda r: int(r[key]))
    marks = [i for i, r in enumerate(rows) if "postprocess" in r["Kernel_Name"]]
    print(f"{len(rows)} rows, {len(marks)} phase markers", file=sys.stderr)
    out = {}
    for k, ph in enumerate(PHASES):
        if 2 * k + 1 < len(marks):
            out[ph] = [r for r in rows[marks[2 * k] + 1:marks[2 * k + 1]] if "clk_kernel" not in r["Kernel_Name"]]
    clk = [r for r in rows if "clk_kernel" in r["Kernel_Name"]]
    return out, clk


def clock_series(samples, clk_rows):
    """{phase: (times_ns, mhz)} from the sampler's samples, placed on the trace's clock."""
    if samples is None or not clk_rows:
        return {}
    names = [p for p in ["idle"] + PHASES if p in samples.files]
    clk_rows = sorted(clk_rows, key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    for name, r in zip(names, clk_rows):
        s = samples[name]
        if len(s) < 3:
            continue
        t0 = int(r["Start_Timestamp"])
        t = [t0 + (int(a) - int(s[0][0])) * 10 for a, _ in s]
        mhz = [(s[i + 1][1] - s[i][1]) / (s[i + 1][0] - s[i][0]) * 100.0 for i in range(len(s) - 1)]
        out[name] = (t[1:], mhz)
    return out


def clock_over(series, a, b):
    t, m = series
    i, j = bisect.bisect_left(t, a), bisect.bisect_right(t, b) + 1
    v = m[i:j]
    return statistics.mean(v) if v else None


def summarize(sel, series):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in sel]
    out = {"launches": len(d), "mean_us": round(statistics.mean(d) / 1e3, 2),
           "median_us": round(statistics.median(d) / 1e3, 2), "min_us": round(min(d) / 1e3, 2),
           "sum_ms": round(sum(d) / 1e6, 3)}
    if series is not None:
        cl = [clock_over(series, int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel]
        ok = [(c, x) for c, x in zip(cl, d) if c is not None]
        if ok:
            out["clock_mhz"] = round(statistics.mean(c for c, _ in ok), 1)
            out["mean_kcycles"] = round(statistics.mean(c * x / 1e6 for c, x in ok), 2)
    return out


def main():
    args = sys.argv[1:]
    samples = pmc = None
    if "--samples" in args:
        import numpy as np
        samples = np.load(args[args.index("--samples") + 1])
    if "--pmc" in args:
        pmc = args[args.index("--pmc") + 1]
    ph, clk = split(rows_of(args[0]), "Start_Timestamp")
    series = clock_series(samples, clk)
    res = {"phase_clock_mhz": {k: round(statistics.median(v[1]), 1) for k, v in series.items()}}
    keys = {p: {(r["Kernel_Name"], grid(r)) for r in ph.get(p, [])} for p in ("proj", "flash")}
    for p, ks in keys.items():
        for where in ("forward", p):
            sel = [r for r in ph.get(where, []) if (r["Kernel_Name"], grid(r)) in ks]
            if sel:
                res[f"{p}@{where}"] = summarize(sel, series.get(where))
                res[f"{p}@{where}"]["kernels"] = sorted({short(k[0]) for k in ks})
    # every family in context vs in the all-GEMM / flash graphs
    for where in ("forward", "gemm", "flash"):
        fams = {}
        for r in ph.get(where, []):
            fams.setdefault(family(r["Kernel_Name"]), []).append(r)
        for f, sel in sorted(fams.items()):
            res[f"family {f}@{where}"] = summarize(sel, series.get(where))
    if pmc:
        disp = {}
        for r in rows_of(pmc):
            d = disp.setdefault(int(r["Dispatch_Id"]), {"Kernel_Name": r["Kernel_Name"], "Grid_Size": grid(r),
                                                        "Dispatch_Id": int(r["Dispatch_Id"])})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
        pph, _ = split(list(disp.values()), "Dispatch_Id")
        for p, ks in keys.items():
            for where in ("forward", p):
                sel = [r for r in pph.get(where, []) if (r["Kernel_Name"], r["Grid_Size"]) in ks]
                hit = sum(r.get("TCC_HIT_sum", 0.0) for r in sel)
                miss = sum(r.get("TCC_MISS_sum", 0.0) for r in sel)
                if sel and hit + miss > 0:
                    e = res.setdefault(f"{p}@{where}", {})
                    e["l2_hit_rate"] = round(hit / (hit + miss), 4)
                    e["l2_miss_per_launch"] = round(miss / len(sel))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
