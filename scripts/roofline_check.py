#!/usr/bin/env python3
"""Cross-check bench.py's live roofline numbers against a rocprofv3 kernel trace of the same command.

Per UNet forward (forwards counted by time_features_kernel<bf16>, launched once per forward):
  bf16 gemm_kernel launches, their summed duration, and the average launch duration; the same for
  flash_attn_d64_kernel.  bench.py reports kernel_ms_per_forward / avg_launch_us from HIP events."""
import csv
import json
import sys


def main(trace, bench_log):
    rows = list(csv.DictReader(open(trace)))
    fwd = sum(1 for r in rows if "time_features_kernel" in r["Kernel_Name"] and "DF16b" in r["Kernel_Name"])
    out = {"forwards_in_trace": fwd}
    for key, pats in (("gemm", ("gemm_kernelIDF16b", "gemm8_kernelIDF16b")), ("flash", ("flash_attn_d64_kernelIDF16b",))):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
             if any(pat in r["Kernel_Name"] for pat in pats)]
        out[key] = {"launches_per_forward": len(d) / fwd, "ms_per_forward": sum(d) / fwd / 1e3,
                    "avg_launch_us": sum(d) / len(d)}
    bench = None
    for line in open(bench_log):
        if line.startswith("{"):
            bench = json.loads(line)
    if bench:
        out["bench"] = {"gemm_ms_per_forward": bench["roofline"]["kernel_ms_per_forward"],
                        "gemm_avg_launch_us": bench["roofline"]["avg_launch_us"],
                        "flash_ms_per_forward": bench["attention"]["ms"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
