#!/usr/bin/env python3
"""The eight-XCD lower bound on the C2 forward's GEMM-family L2-miss traffic, launch by launch.

Each of the 8 XCDs has its own 4 MiB L2, and a launch's tiles are dealt to the XCDs in contiguous chunks. Every XCD
therefore misses at least once on each A row panel and each W column panel its chunk touches. Split a launch's tile
space into a x c XCD rectangles (a * c = 8). Then the reads are at least 8 * (A / a + W / c); the tile walk's group_m
picks the split, so the bound takes the best one. Outputs are written once. This is the bound any XCD-contiguous tile
order has. bench.py's roofline `traffic` compares with it: the measured FETCH_SIZE / WRITE_SIZE over the same forward
is in profiles/*_gemm_traffic.json.

  GPU:  python scripts/gemm_traffic_floor.py --record gpurun_out/<tag>_gemm_launches.json
        (records every GEMM-family launch of one C2 UNet forward: label, algorithmic FLOPs / bytes)
  CPU:  python scripts/gemm_traffic_floor.py --from <launches.json[.gz]> [--traffic profiles/r06l_gemm_traffic.json]

Per launch (bf16 operands, 2 bytes):
  gemm M N K b: A = M K, W = N K, C = M N (N / 2 for geglu), + C again for a residual read
  conv M N K (implicit 3x3, K = 9 Cin): A = M Cin (the activation, not its 9x im2col; M / 4 rows for 'up'), W = N K
  batched launches (b > 1) spread whole batch entries over the XCDs when b >= 8 (no replication).
"""
import argparse
import gzip
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPLITS = [(1, 8), (2, 4), (4, 2), (8, 1)]


def parse(label):
    m = re.match(r"(gemm|conv) M=(\d+) N=(\d+) K=(\d+) b=(\d+) (\S+)(.*)", label or "")
    if not m:
        return None
    kind, M, N, K, b, act, rest = m.groups()
    return dict(kind=kind, M=int(M), N=int(N), K=int(K), b=max(int(b), 1), act=act, up=" up" in rest,
                res=" res" in rest, cat=" cat" in rest)


def floor_of(d, esz=2):
    M, N, K, b = d["M"], d["N"], d["K"], d["b"]
    if d["kind"] == "conv":
        cin = K // 9
        A = (M // 4 if d["up"] else M) * cin * esz
    else:
        A = M * K * esz
    W = N * K * esz
    C = M * (N // 2 if d["act"] == "geglu" else N) * esz
    wr = b * C
    rd_alg = b * (A + W) + (b * C if d["res"] else 0)
    if b >= 8:
        rd_floor = rd_alg
    else:
        per = 8 // b if 8 % b == 0 else 8  # XCDs per batch entry
        opts = [(a, c) for a, c in SPLITS if a * c == per] or [(per, 1), (1, per)]
        rd_floor = b * min(per * (A / a + W / c) for a, c in opts) + (b * C if d["res"] else 0)
    return rd_alg, rd_floor, wr


def record(path):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
    import torch

    import bench
    from fdhip import lib as L
    from fdhip import ops
    L.require_device()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pipe = bench.build_pipe(dev, fp8=False)
    loop = bench.C2Loop(pipe, 1024, 0)
    for i in range(3):
        loop.step(i)
    torch.cuda.synchronize()
    rec = []
    g = torch.cuda.CUDAGraph()
    ops.set_recorder(rec)
    try:
        with torch.cuda.graph(g):
            loop.unet.forward(*loop.args(), cond_embedded=True)
    finally:
        ops.set_recorder(None)
    out = [{"kind": r[0], "flops": r[1], "bytes": r[2], "label": r[4]} for r in rec]
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump({"workload": "C2 1024, one UNet forward (B = 2 CFG rows)", "launches": out}, f)
    print(f"{len(out)} launches recorded -> {path}")
    return path


def report(path, traffic):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        launches = json.load(f)["launches"]
    tot = dict(n=0, rd_alg=0.0, rd_floor=0.0, wr=0.0, flops=0.0, unparsed=0)
    per_shape = {}
    for r in launches:
        if r["kind"] != "gemm":
            continue
        d = parse(r["label"])
        if d is None:
            tot["unparsed"] += 1
            continue
        a, f, w = floor_of(d)
        tot["n"] += 1
        tot["rd_alg"] += a
        tot["rd_floor"] += f
        tot["wr"] += w
        tot["flops"] += r["flops"]
        key = r["label"]
        e = per_shape.setdefault(key, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += a
        e[2] += f
    res = {"launches": tot["n"], "unparsed_launches": tot["unparsed"], "tflop": round(tot["flops"] / 1e12, 3),
           "read_algorithmic_gb": round(tot["rd_alg"] / 1e9, 2), "read_floor_8xcd_gb": round(tot["rd_floor"] / 1e9, 2),
           "write_gb": round(tot["wr"] / 1e9, 2),
           "floor_over_algorithmic": round(tot["rd_floor"] / tot["rd_alg"], 3)}
    if traffic:
        t = json.load(open(traffic))
        rd, wr = t["gemm_read_bytes"], t["gemm_write_bytes"]
        res["measured"] = {"file": os.path.basename(traffic), "launches": t.get("gemm_launches"),
                           "read_gb": round(rd / 1e9, 2), "write_gb": round(wr / 1e9, 2),
                           "read_over_floor": round(rd / tot["rd_floor"], 3),
                           "read_over_algorithmic": round(rd / tot["rd_alg"], 3),
                           "write_over_outputs": round(wr / tot["wr"], 3)}
    top = sorted(per_shape.items(), key=lambda kv: -kv[1][2])[:12]
    res["largest_floors"] = [{"label": k, "launches": v[0], "read_alg_gb": round(v[1] / 1e9, 3),
                              "read_floor_gb": round(v[2] / 1e9, 3)} for k, v in top]
    print(json.dumps(res, indent=1))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--record")
    ap.add_argument("--from", dest="src")
    ap.add_argument("--traffic")
    ap.add_argument("--out")
    a = ap.parse_args()
    src = record(a.record) if a.record else a.src
    if not src:
        ap.error("--record or --from")
    res = report(src, a.traffic)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
