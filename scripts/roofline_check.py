#!/usr/bin/env python3
"""Cross-check bench.py's roofline numbers against the rocprofv3 kernel trace of the same command.

bench.py measures the GEMM family (and flash attention) by replaying the forward's launches of that family as
their own hipGraph between HIP events.  The trace gives, for the same run:
  * in-context: the GEMM / flash kernels of the timed C2 steps (between the first timed fd_tlc_scale_input and
    the last fd_tlc_blend), summed per step -- the family's time inside the real step;
  * family-graph: the same kernels replayed by the family graph, per replay.
frac = algorithmic FLOPs / time / 2500 TFLOP/s is recomputed from each and compared with the bench line.
Usage: roofline_check.py <kernel_trace.csv> <bench.log> [warmup]"""
import csv
import json
import sys

PEAK = 2500.0


def is_gemm(n):
    # rocprofv3 leaves some names mangled (DF16b = bf16) and demangles others (__hip_bfloat16, or the template
    # arguments lost: "conv_halo_kernel<bool _Accum, ...>"); the C2 UNet has no fp16 GEMM / conv launches
    fam = "gemm_kernel" in n or "gemm8_kernel" in n or "gemm256_kernel" in n or "conv_halo_kernel" in n
    return fam and "e4m3" not in n and "DF16_" not in n and "__half" not in n


def main(trace, bench_log, warmup=3):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    starts = [i for i, n in enumerate(names) if "tlc_scale_input" in n]
    blends = [i for i, n in enumerate(names) if "tlc_blend" in n]
    a, b = starts[warmup], blends[-1]
    nsteps = len(starts) - warmup
    bench = None
    for line in open(bench_log):
        if line.startswith("{"):
            bench = json.loads(line)
    rl, at = bench["roofline"], bench.get("attention", {})
    fl_g = rl["algorithmic_flops"]
    out = {"steps_in_window": nsteps}
    for key, pred, flops, bench_ms in (("gemm", is_gemm, fl_g, rl["kernel_ms_per_forward"]),
                                       ("flash", lambda n: "flash_attn_d64" in n, None, at.get("ms_per_forward"))):
        ctx = [dur[i] for i in range(a, b + 1) if pred(names[i])]
        ctx_ms = sum(ctx) / nsteps / 1e3
        # family-graph replays: after the timed window, runs of consecutive same-family launches of the
        # per-forward count
        per_fwd = round(len(ctx) / nsteps)
        tail = [i for i in range(b + 1, len(names)) if pred(names[i])]
        runs, cur = [], []
        for i in tail:
            if cur and i != cur[-1] + 1:
                runs.append(cur)
                cur = []
            cur.append(i)
        if cur:
            runs.append(cur)
        fam = [r[j:j + per_fwd] for r in runs if len(r) % per_fwd == 0 for j in range(0, len(r), per_fwd)]
        fam_ms = sum(sum(dur[i] for i in r) for r in fam) / len(fam) / 1e3 if fam else None
        e = {"launches_per_forward": per_fwd, "in_context_ms_per_step": round(ctx_ms, 4),
             "in_context_avg_launch_us": round(sum(ctx) / len(ctx), 3),
             "family_graph_replays_in_trace": len(fam),
             "family_graph_kernel_sum_ms": None if fam_ms is None else round(fam_ms, 4),
             "bench_event_ms": bench_ms}
        if flops is None and key == "flash":
            flops = at.get("achieved", 0) * 1e12 * (at.get("ms_per_forward", 0) / 1e3)
        if flops:
            e["frac_in_context"] = round(flops / (ctx_ms / 1e3) / 1e12 / PEAK, 4)
            if fam_ms:
                e["frac_family_graph_trace"] = round(flops / (fam_ms / 1e3) / 1e12 / PEAK, 4)
            if bench_ms:
                e["frac_bench"] = round(flops / (bench_ms / 1e3) / 1e12 / PEAK, 4)
                e["bench_vs_in_context"] = round(ctx_ms / bench_ms, 4)
        out[key] = e
    wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e6 / nsteps
    out["step_wall_ms_in_trace"] = round(wall, 3)
    out["bench_ms_per_step"] = bench["ms_per_step"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3)
