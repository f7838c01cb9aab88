"""Host restatement of the OCP MX e4m3 rule the HIP producers share (faithdiff-dev_amd/csrc/fd_common.h mx_exp /
mx_pack4): test infrastructure, used by tests/test_fp8_gpu.py (GPU bytes vs this) and tests/test_mx_rule_cpu.py."""
import torch


def e4m3(x):
    return x.to(torch.float8_e4m3fn).view(torch.uint8)


def mx_ref(x, K=None):
    """Restatement of the MX rule (fd_common.h mx_exp / mx_pack4) on the host: per 32-element block,
    E = least exponent with amax <= 448 * 2^E (amax = ma * 2^ea, ma in [1, 2): E = ea - 8 if ma <= 1.75 else ea - 7;
    all-zero block E = 0), q = RNE_e4m3(x * 2^-E), scale byte = E + 127."""
    x = x.float().cpu()
    M, K = x.shape
    xb = x.reshape(M, K // 32, 32)
    amax = xb.abs().amax(-1)
    m, e = torch.frexp(amax)  # amax = m * 2^e, m in [0.5, 1)
    E = torch.where(2 * m <= 1.75, e - 1 - 8, e - 1 - 7)
    E = torch.where(amax > 0, E, torch.zeros_like(E)).clamp(-127, 127)
    q = e4m3((xb * torch.exp2(-E.float())[..., None]).reshape(M, K))
    return q, (E + 127).to(torch.uint8)
