"""The MX e4m3 scale rule (tests/mx_ref.py, restating fd_common.h mx_exp): E is the LEAST exponent with
amax <= 448 * 2^E -- checked against a brute-force search on random, power-of-two and 1.75 * 2^k block maxima -- so
no element saturates, and dequantization is within e4m3's half ulp.  CPU only (no kernel call)."""
import math

import torch

from mx_ref import mx_ref


def _brute_E(amax):
    if amax == 0.0:
        return 0
    E = -140
    while amax > 448.0 * 2.0 ** E:
        E += 1
    return max(-127, min(127, E))


def test_mx_scale_is_least_exponent_without_saturation():
    g = torch.Generator().manual_seed(0)
    vals = [0.0, 1.0, 448.0, 448.0 * 2 ** 3, 1.75 * 2 ** -5, 1.7500001, 1.7499999, 3.5, 0.001, 12345.678, 2.0 ** -100]
    vals += (torch.rand(200, generator=g) * torch.logspace(-20, 20, 200)).tolist()
    x = torch.zeros(len(vals), 32)
    for i, v in enumerate(vals):
        x[i, 0] = v
        x[i, 1:] = torch.rand(31, generator=g) * v
    q, s = mx_ref(x)
    for i, v in enumerate(vals):
        amax = float(x[i].abs().max())
        assert int(s[i, 0]) - 127 == _brute_E(amax), (v, amax)
    deq = q.view(torch.float8_e4m3fn).float() * torch.exp2(s.float() - 127).repeat_interleave(32, 1)
    assert torch.isfinite(deq).all()
    blk = torch.exp2(s.float() - 127).repeat_interleave(32, 1)
    assert torch.all((deq - x).abs() <= x.abs() * 2.0 ** -4 + blk * 2.0 ** -10)
    assert math.isclose(float(deq.abs().max()), float(x.abs().max()), rel_tol=2.0 ** -4)
