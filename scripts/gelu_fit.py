#!/usr/bin/env python3
"""The GELU form of the GEMM epilogues (csrc/fd_common.h gelu_f): GELU(x) = x * Phi(x) = x * sigmoid(z(x)) with
z = logit(Phi(x)), an odd function, fitted as x * (c0 + c1 x^2 + c2 x^4) on |x| <= 5.5 (x clamped there: beyond it
Phi(x) is 0 or 1 to within 2e-8) by Lawson-reweighted least squares on the GELU error x * Phi (1 - Phi) * dz.
Prints the coefficients with -log2(e) folded in (the kernel computes 1 / (1 + exp2(p))) and the max |error| against
the exact x * Phi(x) in float64 and in a float32 emulation of the kernel's operation order.

    python scripts/gelu_fit.py
"""
import numpy as np
from scipy.stats import norm


def fit(deg=3, lim=5.5, iters=300):
    xs = np.linspace(1e-3, lim, 40000)
    phi = norm.cdf(xs)
    z = norm.logcdf(xs) - norm.logcdf(-xs)
    w0 = xs * phi * (1 - phi)
    A = np.stack([xs ** (2 * k + 1) for k in range(deg)], 1)
    w = w0.copy()
    for _ in range(iters):
        c, *_ = np.linalg.lstsq(A * np.sqrt(w)[:, None], z * np.sqrt(w), rcond=None)
        e = np.abs((A @ c - z) * w0)
        w = w * (e / e.max() + 1e-12)
        w /= w.sum()
    return c


def main():
    lim = 5.5
    c = fit(3, lim)
    k = -c * np.log2(np.e)
    x = np.linspace(-12, 12, 2400001)
    exact = x * norm.cdf(x)
    xc = np.clip(x, -lim, lim)
    p = (k[2] * xc ** 2 + k[1]) * xc ** 2 + k[0]
    g = x / (1 + np.exp2(p * xc))
    f = np.float32
    x32, k32 = x.astype(f), k.astype(f)
    xc32 = np.clip(x32, f(-lim), f(lim))
    x2 = xc32 * xc32
    p32 = ((k32[2] * x2 + k32[1]) * x2 + k32[0]) * xc32  # fp32 (the kernel's fmas round once less)
    g32 = x32 * (f(1) / (f(1) + np.exp2(p32)))
    print("coefficients (times -log2 e):", ", ".join(f"{v:.9e}f" for v in k.astype(np.float32)))
    print(f"max |err| float64 {np.abs(g - exact).max():.3e}, float32 {np.abs(g32.astype(np.float64) - exact).max():.3e}")


if __name__ == "__main__":
    main()
