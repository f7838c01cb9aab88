"""Measured parity metrics of the GPU tests (rel-L2, cosine, PSNR, max-rel), recorded under the running test's id
and written when the session ends to $FD_PARITY_METRICS (default gpurun_out/parity_metrics.json; copied per round to
profiles/rNN_parity_metrics.json) -- the measured numbers behind DESIGN.md section 3's bars.  Test infrastructure
only (tests/conftest.py sets the current test and writes the file)."""
import json
import math
import os

CURRENT = {"test": None}
RECORDS = {}


def record(name, value, bar=None):
    """Record one measured metric of the running test (bar: the threshold the test asserts, when given)."""
    ent = {"metric": name, "value": float(value)}
    if bar is not None:
        ent["bar"] = bar
    RECORDS.setdefault(CURRENT["test"] or "<no test>", []).append(ent)
    return value


def rel_l2(a, b, name="rel_l2"):
    a, b = a.double(), b.double()
    return record(name, ((a - b).norm() / b.norm().clamp_min(1e-30)).item())


def maxrel(a, b):
    a, b = a.float(), b.float()
    return record("max_rel", ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item())


def cos(a, b):
    import torch
    return record("cos", torch.nn.functional.cosine_similarity(a.double().flatten(), b.double().flatten(), dim=0).item())


def psnr(a, b, peak, name="psnr_db"):
    import numpy as np
    mse = float(((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2).mean())
    return record(name, 99.0 if mse == 0 else 10 * math.log10(peak ** 2 / mse))


def dump(path=None):
    if not RECORDS:
        return None
    default = "parity_metrics.json"
    try:  # a CPU-only run (no device) writes its own file, never over a GPU run's merged metrics
        import torch
        if not torch.cuda.is_available():
            default = "parity_metrics_cpu.json"
    except ImportError:
        default = "parity_metrics_cpu.json"
    path = path or os.environ.get("FD_PARITY_METRICS") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "gpurun_out", default)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump({"tests": len(RECORDS), "metrics": RECORDS}, f, indent=1, sort_keys=True)
    return path
