#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of scripts/incontext_probe.py into its phases (fd_postprocess_u8 markers) and
compare the same launches in context (the forward graph) and in their family graphs: per (kernel, grid) the count
per replay and the mean / median / min duration, in each phase.  With a PMC trace of TCC_HIT_sum / TCC_MISS_sum
(second argument) it adds the L2 hit rate of those launches in each phase.

    python scripts/incontext_report.py <kernel_trace.csv> [<counter_collection.csv>] > out.json
"""
import csv
import json
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

PHASES = ["forward", "proj", "flash", "gemm"]


def phases_of(rows, key_start, key_name):
    rows = sorted(rows, key=lambda r: int(r[key_start]))
    marks = [i for i, r in enumerate(rows) if "postprocess_u8" in r[key_name]]
    # markers come in pairs around each phase's replays, in PHASES order
    out = {}
    for k, ph in enumerate(PHASES):
        if 2 * k + 1 < len(marks):
            out[ph] = rows[marks[2 * k] + 1:marks[2 * k + 1]]
    return out


def grid(r):
    return int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)


def fam(name):
    if "flash_attn_d64" in name:
        return "flash_d64"
    if "gemm_kernel" in name:
        return "gemm4w"
    return None


def main():
    trace = list(csv.DictReader(open(sys.argv[1])))
    ph = phases_of(trace, "Start_Timestamp", "Kernel_Name")
    res = {}
    # the (kernel, grid) keys of the family phases
    keys = {"proj": set(), "flash": set()}
    for p in keys:
        for r in ph.get(p, []):
            keys[p].add((r["Kernel_Name"], grid(r)))
    for p, ks in keys.items():
        for where in ("forward", p):
            d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ph.get(where, [])
                 if (r["Kernel_Name"], grid(r)) in ks]
            if d:
                res[f"{p}@{where}"] = {"launches": len(d), "mean_us": round(statistics.mean(d) / 1e3, 2),
                                       "median_us": round(statistics.median(d) / 1e3, 2),
                                       "min_us": round(min(d) / 1e3, 2), "sum_ms": round(sum(d) / 1e6, 3),
                                       "kernels": sorted({short(k[0]) for k in ks})}
    if len(sys.argv) > 2:
        pm = list(csv.DictReader(open(sys.argv[2])))
        disp = {}
        for r in pm:
            d = disp.setdefault(int(r["Dispatch_Id"]), {"Kernel_Name": r["Kernel_Name"],
                                                        "Grid_Size": grid(r),
                                                        "Dispatch_Id": int(r["Dispatch_Id"])})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
        pph = phases_of(list(disp.values()), "Dispatch_Id", "Kernel_Name")
        for p, ks in keys.items():
            for where in ("forward", p):
                sel = [r for r in pph.get(where, []) if (r["Kernel_Name"], r["Grid_Size"]) in ks]
                hit = sum(r.get("TCC_HIT_sum", 0.0) for r in sel)
                miss = sum(r.get("TCC_MISS_sum", 0.0) for r in sel)
                if sel and hit + miss > 0:
                    res.setdefault(f"{p}@{where}", {})["l2_hit_rate"] = round(hit / (hit + miss), 4)
                    res[f"{p}@{where}"]["l2_miss_per_launch"] = round(miss / len(sel))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
