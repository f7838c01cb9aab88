#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of scripts/prof.sh over one scripts/pmc_work.py workload.

Input: <dir>/{trace,FETCH_SIZE,WRITE_SIZE,sq1,sq2,...}/**.csv + meta.json (dir default gpurun_out/pmc_<what>).  The measured window
is the dispatches between the last two fd_postprocess_u8 markers; the calibration copy sits between the two
before.  Per kernel family: launches, summed durations from the trace-only pass (profiled PMC passes run slower,
so durations never come from them), HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB; gfx950 FETCH_SIZE counts half
of a 16-B/lane streaming read, MI355X_MICROARCH.md HBM section; the calibration copy's measured bytes/count is
recorded beside it), achieved GB/s and TFLOP/s, and every SQ counter summed over the family's dispatches, with
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMD x 256 CU x GRBM_GUI_ACTIVE / 8 XCD).
Usage: pmc_report.py <what> <out.json> [dir]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def family(name):
    # e4m3 operands: the 4-wave kernels, and gemm8 instantiated on uint8_t (per-row) / mx8_t (MX) operands
    if "gemm_e4m3" in name or "gemm8_kernelIh" in name or "gemm8_kernelI5mx8_t" in name:
        return "gemm_e4m3"
    if "gemm_kernel" in name or "gemm8_kernel" in name or "gemm256_kernel" in name or "conv_halo_kernel" in name:
        return "gemm"
    if "quant_rows_e4m3" in name or "layer_norm_e4m3" in name:
        return "fp8_quant"
    if "flash_attn" in name:
        return "flash_attn"
    if "gn_" in name:
        return "group_norm"
    if "softmax" in name:
        return "softmax"
    return "other"


def window(seq):
    marks = [i for i, n in enumerate(seq) if "postprocess_kernel" in n]
    m1, m2, m3 = marks[-3:]
    return (m1 + 1, m2), (m2 + 1, m3)


def load_trace(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    return [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]


def load_counters(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None
    per = defaultdict(lambda: [None, defaultdict(float)])
    for r in csv.DictReader(open(f[0])):
        e = per[int(r["Dispatch_Id"])]
        e[0] = r["Kernel_Name"]
        e[1][r["Counter_Name"]] += float(r["Counter_Value"])
    return [(per[k][0], dict(per[k][1])) for k in sorted(per)]


def main(what, out_path, base=None):
    base = base or os.path.join(ROOT, "gpurun_out", f"pmc_{what}")
    meta = json.load(open(os.path.join(base, "meta.json")))
    tr = load_trace(os.path.join(base, "trace"))
    (c0, c1), (w0, w1) = window([n for n, _ in tr])
    fams = defaultdict(lambda: {"launches": 0, "us": 0.0, "counters": defaultdict(float)})
    for n, us in tr[w0:w1]:
        f = fams[family(n)]
        f["launches"] += 1
        f["us"] += us
    res = {"workload": meta["workload"], "window_us": sum(us for _, us in tr[w0:w1]),
           "calibration_copy_us": sum(us for _, us in tr[c0:c1])}
    calib = {}
    seen = set()
    for p in sorted(os.listdir(base)):
        d = os.path.join(base, p)
        if p == "trace" or not os.path.isdir(d):
            continue
        cs = load_counters(d)
        if cs is None:
            continue
        (a0, a1), (b0, b1) = window([n for n, _ in cs])
        # a counter collected in several passes (GRBM_GUI_ACTIVE rides along with each SQ group) is taken
        # from the first pass only; the same pass's own kernel trace gives the durations its clock refers to
        pass_names = set(k for _, vals in cs for k in vals)
        fresh = pass_names - seen
        seen |= pass_names
        ptr = load_trace(d)
        (_, _), (pw0, pw1) = window([n for n, _ in ptr])
        pdur = defaultdict(float)
        for n, us in ptr[pw0:pw1]:
            pdur[family(n)] += us
        for n, vals in cs[b0:b1]:
            for k, v in vals.items():
                if k in fresh:
                    fams[family(n)]["counters"][k] += v
        if "GRBM_GUI_ACTIVE" in fresh:
            for fn_, us in pdur.items():
                fams[fn_]["grbm_pass_us"] = us
        for n, vals in cs[a0:a1]:
            for k, v in vals.items():
                if k in fresh:
                    calib[k] = calib.get(k, 0.0) + v
    out = {}
    for name, f in sorted(fams.items(), key=lambda x: -x[1]["us"]):
        c = f["counters"]
        e = {"launches": f["launches"], "ms": round(f["us"] / 1e3, 4)}
        m = meta["families"].get(name)
        if m:
            e.update(algorithmic_flops=m["flops"], algorithmic_bytes=m["algorithmic_bytes"])
            if m["flops"]:
                e["achieved_tflops"] = round(m["flops"] / (f["us"] / 1e6) / 1e12, 1)
            if m["algorithmic_bytes"]:
                e["algorithmic_gbs"] = round(m["algorithmic_bytes"] / (f["us"] / 1e6) / 1e9, 1)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rd, wr = 2 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
            e.update(hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_gbs=round((rd + wr) / (f["us"] / 1e6) / 1e9, 1))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"]:
            e["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * 256 * c["GRBM_GUI_ACTIVE"] / 8), 4)
            if f.get("grbm_pass_us"):
                # GRBM_GUI_ACTIVE / 8 / wall reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md,
                # DVFS give-back), so mfma_busy above is a lower bound; the bound below assumes the 2.4 GHz peak clock
                e["effective_clock_ghz_profiled"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (f["grbm_pass_us"] * 1e3), 3)
                e["mfma_busy_at_2p4ghz"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * 2.4e3 * f["grbm_pass_us"]), 4)
        e["counters"] = {k: v for k, v in sorted(c.items())}
        out[name] = e
    res["families"] = out
    # per-launch table of the timed kinds, in launch order (labels recorded by pmc_work.py)
    labs = [x for x in meta.get("labels", []) if x[0] in ("gemm", "gemm_e4m3", "flash_attn", "group_norm")]
    timed = [(n, us) for n, us in tr[w0:w1] if family(n) in ("gemm", "gemm_e4m3", "flash_attn", "group_norm")
             and "gn_partial" not in n and "gn_finalize" not in n]
    if labs and len(labs) == len(timed):
        res["launches"] = [{"kind": k, "label": lab, "us": round(us, 2),
                            "tflops": round(fl / (us / 1e6) / 1e12, 1) if fl else None}
                           for (k, lab, fl), (n, us) in zip(labs, timed)]
    if "FETCH_SIZE" in calib:
        res["calibration"] = {"bytes_read": meta["calib_bytes_read"], "bytes_written": meta["calib_bytes_written"],
                              "fetch_kib_x2": 2 * calib["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in calib else None,
                              "write_kib": calib.get("WRITE_SIZE", 0) * 1024}
    res["method"] = ("scripts/prof.sh: rocprofv3 --kernel-trace (durations) and separate --pmc passes "
                     "(FETCH_SIZE; WRITE_SIZE; SQ groups) over scripts/pmc_work.py --what " + what)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "counters"} for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
