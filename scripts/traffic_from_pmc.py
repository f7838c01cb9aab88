#!/usr/bin/env python3
"""bench.py's roofline.traffic file from a UNet PMC report (scripts/prof.sh unet <tag> -> gpurun_out/<tag>.json; scripts/run.sh <tag> pmc=unet runs it on the box): the GEMM
family's memory-side bytes per forward, read = 2 x FETCH_SIZE KiB (gfx950 counts 16-B/lane reads at half),
write = WRITE_SIZE KiB, with the report's 1 GiB calibration copy alongside.
Usage: traffic_from_pmc.py <unet pmc json> <out json> [family: gemm (default) | gemm_e4m3]"""
import json
import os
import sys


def main(src, dst, family="gemm"):
    r = json.load(open(src))
    g = r["families"][family]
    out = {"workload": r["workload"].replace(" UNet forward", ""),  # the key bench.load_traffic matches
           "source": ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) + --kernel-trace over "
                      "scripts/pmc_work.py --what unet (scripts/prof.sh unet <tag>, scripts/pmc_report.py, scripts/traffic_from_pmc.py); profiles/"
                      + os.path.basename(src)),
           "family": family, "gemm_launches": g["launches"], "gemm_read_bytes": g["hbm_read_bytes"],
           "gemm_write_bytes": g["hbm_write_bytes"],
           "hbm_bytes_per_forward": g["hbm_read_bytes"] + g["hbm_write_bytes"],
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count of 16-B/lane reads), write = WRITE_SIZE KiB",
           "calibration": r.get("calibration")}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:4])
