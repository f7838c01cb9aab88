"""Tensor-level wrappers over the C ABI.  Tensors are device buffers only; all arithmetic is HIP.

Layout conventions: activations NHWC, flattened to [M, C] with M = n*H*W; Linear weights [N, K];
3x3 conv weights pre-packed [Cout, 9*Cin] (tap-major, see pack_conv3x3).
"""
import ctypes
import weakref

import torch

from . import knobs
from . import lib as L

_GN_WS = {}
# Workspace lifetime: a hipGraph captured while a workspace buffer was current keeps its address and writes there
# on every replay.  GraphCache therefore holds a reference to every live workspace (live_workspaces()) in each
# entry it captures; when a workspace grows here, the old buffer is dropped from this module and stays allocated
# exactly as long as some graph captured against it is alive.  Workspaces never grow inside a capture (the graph
# cache runs every shape eagerly first, which sizes them), and they grow geometrically (2x).


def live_workspaces():
    """The current GroupNorm and split-K workspace buffers (GraphCache keeps them alive with a captured graph)."""
    return list(_GN_WS.values()) + list(_GEMM_WS.values())


def _gn_ws(nbytes, device):
    key = device
    ws = _GN_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"GroupNorm workspace too small inside graph capture ({nbytes} B): run the shape "
                               "once eagerly or call ops.reserve_gn_workspace first")
        grow = 0 if ws is None else 2 * ws.numel()
        ws = torch.empty(max(nbytes, grow, 1 << 20), dtype=torch.uint8, device=device)
        _GN_WS[key] = ws
    return ws


def reserve_gn_workspace(nbytes, device):
    """Pre-size the GroupNorm workspace (call before hipGraph capture)."""
    _gn_ws(nbytes, device)


# --------------------------------------------------------------------------------------- GEMM workspace
_GEMM_WS = {}
_ALL_GEMM_WS = weakref.WeakSet()  # every split-K workspace still alive (the current ones and those graphs hold)
_TILE_GROUPS = [1]


class tile_groups:
    """Context: the current forward batches ``n`` TLC tiles along M.  fd_gemm derives its split-K count
    from the per-tile row count (m_ref = M / n), so a batched forward is bitwise equal to per-tile ones."""

    def __init__(self, n):
        self.n = max(int(n), 1)

    def __enter__(self):
        _TILE_GROUPS.append(self.n)
        return self

    def __exit__(self, *exc):
        _TILE_GROUPS.pop()


def reserve_gemm_workspace(nbytes, device):
    """Pre-size the split-K workspace (zeroed: its head holds the tile counters).  Call before capture.  A graph
    captured with the old buffer keeps it alive (GraphCache entries hold live_workspaces()); its counters stay
    zero between launches (the last arriver of every tile resets its counter)."""
    key = torch.device(device)
    ws = _GEMM_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        grow = 0
        if ws is not None:
            torch.cuda.synchronize(key)
            grow = 2 * ws.numel()
        _GEMM_WS[key] = torch.zeros(max(nbytes, grow, 1 << 20), dtype=torch.uint8, device=key)
        _ALL_GEMM_WS.add(_GEMM_WS[key])
    return _GEMM_WS[key]


_SK_HEAD = 65536 * 4  # tile counters + flags at the head of a split-K workspace


def split_k_health(raise_on_timeout=True):
    """Check the pairwise split-K hand-offs (fd_splitk_health; a host sync).  A timed-out wait poisoned its tile with
    NaN and left that tile's counter / flag slot stale, so on any timeout every live split-K workspace's counter
    head is re-zeroed (later launches start clean) and, by default, RuntimeError is raised: the outputs computed
    since the last check are not to be trusted.  Returns the timeout count."""
    n = ctypes.c_uint(0)
    L.check(L.load().fd_splitk_health(ctypes.byref(n), 1), "fd_splitk_health")
    if n.value:
        torch.cuda.synchronize()
        for ws in list(_ALL_GEMM_WS):
            ws[:_SK_HEAD].zero_()
        torch.cuda.synchronize()
        if raise_on_timeout:
            raise RuntimeError(f"{n.value} split-K hand-off wait(s) timed out: the affected tiles were poisoned with "
                               "NaN; the split-K counters have been reset")
    return n.value


def _attach_ws(p, device):
    groups = _TILE_GROUPS[-1]
    p.m_ref = p.M // groups if groups > 1 and p.M % groups == 0 else p.M
    need = L.load().fd_gemm_ws_bytes(ctypes.byref(p))
    if need <= 0:
        return
    key = torch.device(device)
    ws = _GEMM_WS.get(key)
    if ws is None or ws.numel() < need:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"fd_gemm split-K workspace too small inside graph capture ({need} B): "
                               "run the forward once eagerly or call ops.reserve_gemm_workspace first")
        ws = reserve_gemm_workspace(need, device)
    p.ws, p.ws_bytes = ws.data_ptr(), ws.numel()


# --------------------------------------------------------------------------------------- packing
def pack_conv3x3(w):
    """[Cout, Cin, 3, 3] -> [Cout, 9*Cin] with k = (ky*3 + kx)*Cin + c (tap-major, channel-contiguous)."""
    co, ci, kh, kw = w.shape
    return w.permute(0, 2, 3, 1).reshape(co, kh * kw * ci).contiguous()


# taps of a 3x3 kernel on the nearest-x2 upsampled grid that land on source row (col) offset r in {0, 1} of phase a:
# phase 0 (even output rows): r = 0 <- ky 0, r = 1 <- ky 1, 2; phase 1 (odd): r = 0 <- ky 0, 1, r = 1 <- ky 2
_UP2_TAPS = (((0,), (1, 2)), ((0, 1), (2,)))


def pack_conv3x3_up2(w):
    """Upsample2D's conv (nearest x2, then 3x3 pad 1) as four 2x2 phase convs of the low-resolution input:
    [Cout, Cin, 3, 3] -> [4 * Cout, 4 * Cin], row ph * Cout + o (ph = 2a + b: output pixel (2i + a, 2j + b)),
    column (2 ry + rx) * Cin + c: the sum in fp32 of the taps landing on source pixel (i + a - 1 + ry, j + b - 1 + rx)
    (fd_gemm_params.up_phase).  Cast to the conv dtype by the caller (one rounding of each summed weight)."""
    co, ci, _, _ = w.shape
    w = w.float()
    out = torch.zeros(4, co, 2, 2, ci, dtype=torch.float32)
    for a in range(2):
        for b in range(2):
            for ry in range(2):
                for rx in range(2):
                    acc = torch.zeros(co, ci, dtype=torch.float32)
                    for ky in _UP2_TAPS[a][ry]:
                        for kx in _UP2_TAPS[b][rx]:
                            acc += w[:, :, ky, kx].cpu()
                    out[2 * a + b, :, ry, rx, :] = acc
    return out.reshape(4 * co, 4 * ci).contiguous()


def pack_geglu(w, b):
    """GEGLU proj [2F, K] -> rows interleaved in groups of 32 = [16 hidden | 16 gate] (fd_gemm GEGLU)."""
    F2, K = w.shape
    F = F2 // 2
    h, g = w[:F].reshape(F // 16, 16, K), w[F:].reshape(F // 16, 16, K)
    wp = torch.stack([h, g], dim=1).reshape(F2, K).contiguous()
    bh, bg = b[:F].reshape(F // 16, 16), b[F:].reshape(F // 16, 16)
    bp = torch.stack([bh, bg], dim=1).reshape(F2).contiguous()
    return wp, bp


# --------------------------------------------------------------------------------------- GEMM / conv
_probe = None
_recorder = None


def set_probe(records):
    """Measurement hook (per-launch event probe, never on in timed steps): while ``records`` is a list, every
    GEMM / conv (fd_gemm), flash-attention, GroupNorm and LayerNorm launch appends
    (kind, algorithmic FLOPs, algorithmic HBM bytes, start event, end event) recorded on the launch stream.
    None turns it off."""
    global _probe
    _probe = records


def set_recorder(records):
    """Measurement hook for bench.py's kernel-family graphs: while ``records`` is a list, every timed-kind
    launch also appends (kind, algorithmic FLOPs, algorithmic HBM bytes, relaunch, label), where relaunch()
    issues the identical launch again (same parameters and buffers).  Used while a whole forward is being
    captured into a hipGraph, so the buffers are that graph's and stay allocated while it lives; bench.py then
    captures the relaunches of ONE kind (e.g. every GEMM of the forward) into a second graph and times it with
    HIP events.  None turns it off."""
    global _recorder
    _recorder = records


def _timed(kind, flops, nbytes, launch, label=None):
    if _recorder is not None:
        _recorder.append((kind, float(flops), float(nbytes), launch, label))
    if _probe is None:
        launch()
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    launch()
    e1.record()
    _probe.append((kind, float(flops), float(nbytes), e0, e1) + ((label,) if label else ()))


def _gemm_bytes(p):
    """Algorithmic HBM bytes of one fd_gemm launch: every operand once (A -- for a conv the source image(s), not the
    9x im2col --, B per distinct weight slot, C, the residual), no re-reads (bench.py roofline.algorithmic_bytes)."""
    es = 4 if p.dtype == L.dtype_code(torch.float32) else 2
    eo = {L.dtype_code(torch.float32): 4}.get(p.out_dtype, 2)
    nb = max(p.batch, 1)
    nout = p.N // 2 if p.act == L.ACT["geglu"] else p.N
    a = (p.nimg * p.Hin * p.Win * p.Cin * es) if p.conv else p.M * p.K * es * nb
    slots = nb if p.strideB else 1
    if p.bsel_rows > 0:
        groups = -(-p.M // p.bsel_rows)
        slots = min(groups, p.bsel_mod) if p.bsel_mod > 0 else groups
    b = p.N * p.K * es * slots
    c = p.M * nout * eo * nb * (2 if p.residual else 1)
    return float(a + b + c)


def _launch_gemm(p, what):
    flops = 2.0 * p.M * p.N * p.K * max(p.batch, 1)
    label = None
    nbytes = 0.0
    if _recorder is not None:
        nbytes = _gemm_bytes(p)
    if _probe is not None or _recorder is not None:
        act = {v: k for k, v in L.ACT.items()}[p.act]
        label = (f"{'conv' if p.conv else 'gemm'} M={p.M} N={p.N} K={p.K} b={p.batch} {act}"
                 f"{' up' if p.upsample else ''}{' cat' if p.A2 else ''}{' res' if p.residual else ''}")
    _timed("gemm", flops, nbytes, lambda: L.check(L.load().fd_gemm(ctypes.byref(p), L.stream()), what), label)


class GnStats:
    """GroupNorm statistics asked of the GEMM / conv that produces the GroupNorm's input (fd_gemm_params.gn_part):
    pass it as ``gn=`` to gemm / conv3x3 and as ``stats=`` to group_norm.  ``done`` / ``rows`` are set at launch
    when the chosen kernel wrote them (256-row tiles of gemm8 / gemm256 or the 4-wave kernel's 128 x 128 tiles,
    group-aligned, H*W a multiple of the block rows); otherwise group_norm computes its own.
    The decision depends only on shapes, so it is the same in every replay of a captured graph."""

    def __init__(self, nimg, HW, groups, device):
        self.nimg, self.HW, self.groups = nimg, HW, groups
        # sized for 128-row blocks (the 4-wave kernel's 128 x 128 tiles); 256-row kernels use half of it
        self.part = torch.empty((max(nimg * (HW // 128) * groups * 2, 2),), dtype=torch.float32, device=device)
        self.done, self.rows = False, 0

    def attach(self, p):
        self.done, self.rows = False, 0
        if self.HW % 128 == 0 and p.M == self.nimg * self.HW:
            p.gn_part, p.gn_groups, p.gn_hw = self.part.data_ptr(), self.groups, self.HW

    def collect(self, p):
        self.rows = int(p.gn_done) if p.gn_part else 0  # rows per partial block (256 / 128), 0 = not written
        self.done = self.rows > 0


def _rows(t, ld, ncols):
    """Rows r of ``ld`` elements whose first ``ncols`` elements (the launch's columns) all lie inside t's own extent:
    r * ld + ncols - 1 <= span - 1 (fd_gemm_params.*_rows).  A view whose last row is shorter than the launch's
    columns does not count that row (the first-element count let such a row pass the extent check)."""
    span = 1 + sum((n - 1) * st for n, st in zip(t.shape, t.stride()) if n > 0)
    if t.numel() == 0 or ld <= 0 or ncols <= 0 or span < ncols:
        return 0
    return (span - ncols) // ld + 1


def gemm(a, w, out=None, bias=None, residual=None, rowbias=None, rows_per_group=1, alpha=1.0, act="none",
         out_dtype=None, batch=1, M=None, N=None, K=None, lda=None, ldw=None, ldc=None, ldr=None,
         stride_a=0, stride_w=0, stride_c=0, stride_r=0, ln_out=None, ln_in=None, ln_c=None, ln_eps=1e-5, gn=None,
         batch_inner=1, stride_a_o=0, stride_w_o=0, stride_c_o=0, bsel=None, sm_len=None):
    """out[M, N (N/2 for geglu)] = epi(alpha * a[M, K] @ w[N, K]^T); strides default to the tensors'.
    ln_out: fp32 [M, N/160, 2] -- also write per-row (sum, sumsq) partials of the stored output (LayerNorm
    producer).  ln_in / ln_c: fold LayerNorm(a) into this GEMM (w = W * gamma, ln_c = rowsum(w), bias =
    W . beta + b; see fold_layer_norm).
    batch_inner > 1: two-level batch, operand offsets (z % batch_inner) * stride_x + (z // batch_inner) * stride_x_o.
    bsel = (rows, mod, stride_w, stride_n): rows [g*rows, (g+1)*rows) multiply w + s * stride_w (ln_c / bias +
    s * stride_n), s = g % mod (mod > 0) or g.  act="softmax" with sm_len: softmax over the first sm_len columns of
    every 80-column group of the epilogue (the rest 0) -- fd_gemm_params.sm_* (include/faithdiff_hip.h)."""
    K = a.shape[-1] if K is None else K
    N = w.shape[-2] if N is None else N
    ldw = w.stride(-2) if ldw is None else ldw
    lda = a.stride(-2) if lda is None else lda
    M = (a.numel() // a.shape[-1]) // batch if M is None else M
    nout = N // 2 if act == "geglu" else N
    odt = out_dtype or (out.dtype if out is not None else a.dtype)  # a given out buffer fixes the output type
    if out is None:
        out = torch.empty((batch, M, nout) if batch > 1 else (M, nout), dtype=odt, device=a.device)
    elif out.dtype != odt:
        raise ValueError(f"gemm: out dtype {out.dtype} != out_dtype {odt}")
    p = L.GemmParams()
    p.A, p.B, p.C = a.data_ptr(), w.data_ptr(), out.data_ptr()
    p.lda, p.ldb = lda, ldw
    p.ldc = out.stride(-2) if ldc is None else ldc
    p.strideA, p.strideB, p.strideC = stride_a, stride_w, stride_c
    p.M, p.N, p.K, p.batch = M, N, K, batch
    p.bias = bias.data_ptr() if bias is not None else None
    if residual is not None:
        p.residual = residual.data_ptr()
        p.ldr = residual.stride(-2) if ldr is None else ldr
        p.strideR = stride_r
        p.residual_rows = _rows(residual, p.ldr, N // 2 if act == "geglu" else N)
    if rowbias is not None:
        p.rowbias, p.rowbias_ld = rowbias.data_ptr(), rowbias.stride(0)
        p.rowbias_rows = _rows(rowbias, p.rowbias_ld, N // 2 if act == "geglu" else N)
    p.rows_per_group = rows_per_group
    p.alpha = alpha
    p.act = L.ACT[act]
    p.dtype = L.dtype_code(a.dtype)
    p.out_dtype = L.dtype_code(odt)
    if ln_out is not None:
        p.ln_out = ln_out.data_ptr()
    if ln_in is not None:
        p.ln_in, p.ln_c, p.ln_eps = ln_in.data_ptr(), ln_c.data_ptr(), ln_eps
    if gn is not None and batch == 1:
        gn.attach(p)
    if batch_inner > 1:
        p.batch_inner, p.strideA_o, p.strideB_o, p.strideC_o = batch_inner, stride_a_o, stride_w_o, stride_c_o
    if bsel is not None:
        p.bsel_rows, p.bsel_mod, p.bsel_strideB, p.bsel_strideN = bsel
    if act == "softmax":
        p.sm_group, p.sm_len = 80, int(sm_len)
    _attach_ws(p, a.device)
    _launch_gemm(p, "fd_gemm")
    if gn is not None:
        gn.collect(p)
    return out


XSLOT = 80  # keys per head group of the two-GEMM cross-attention (two heads per 160-column score tile)


class XAttnMats:
    """The per-prompt matrices of one attn2 block for cross-attention as two GEMMs (R prompt rows, C channels, H
    heads of 64): b1 [R, H*80, C] = 0.125 K_r,h W_q' (score matrix, rows h*80 + j), c / d [R, H*80] its LayerNorm-fold
    constants, b2 [R, C, KP] with b2[r][n][h*80 + j] = W_o[n, h] . V_r[j, h] (KP = H*80 rounded up to 64).  Pad rows
    and columns (keys j >= Lk, K past H*80) are zero: allocated zeroed, never written."""

    def __init__(self, R, C, H, dtype, device):
        self.R, self.C, self.H = R, C, H
        self.HP = H * XSLOT
        self.KP = (self.HP + 63) // 64 * 64
        self.b1 = torch.zeros((R, self.HP, C), dtype=dtype, device=device)
        self.c = torch.empty((R, self.HP), dtype=torch.float32, device=device)
        self.d = torch.empty((R, self.HP), dtype=torch.float32, device=device)
        self.b2 = torch.zeros((R, C, self.KP), dtype=dtype, device=device)


def xattn_prepare(m, k, v, ldkv, Lk, wq_t, dq, wo, scale=0.125):
    """Fill XAttnMats m from the prompt keys / values of one block: k, v views whose row r*Lk + j (stride ldkv) is
    prompt r's key / value j (heads at columns h*64); wq_t = W_q'^T [C, C] (W_q' = W_q diag(gamma2) of the folded
    norm2), dq = W_q . beta2 fp32 [C], wo = W_o [C, C].  Three launches, once per prompt."""
    R, C, H, HP, KP, S = m.R, m.C, m.H, m.HP, m.KP, XSLOT
    if Lk > S:
        raise ValueError(f"xattn_prepare: {Lk} keys > {S} per head group")
    # b1: out[j][k] = scale sum_d K_r[j][h*64 + d] W_q'^T[k][h*64 + d], batched over (r, h)
    gemm(k, wq_t, out=m.b1, M=Lk, N=C, K=64, lda=ldkv, ldw=C, ldc=C, alpha=scale, batch=R * H, batch_inner=H,
         stride_a=64, stride_a_o=Lk * ldkv, stride_w=64, stride_w_o=0, stride_c=S * C, stride_c_o=HP * C)
    xattn_consts(m.b1, R * HP, C, k, ldkv, Lk * ldkv, dq, H, S, Lk, scale, m.c, m.d)
    # b2: out[n][h*80 + j] = sum_d W_o[n][h*64 + d] V_r[j][h*64 + d], batched over (r, h)
    gemm(wo, v, out=m.b2, M=C, N=Lk, K=64, lda=C, ldw=ldkv, ldc=KP, batch=R * H, batch_inner=H, stride_a=64,
         stride_a_o=0, stride_w=64, stride_w_o=Lk * ldkv, stride_c=S, stride_c_o=C * KP)


def xattn_attend(h, st, m, P, rows_per_img, mod, s0, Lk, bias_o, st_out=None):
    """h += attn2(LN2(h)) in place, as two GEMMs: P = softmax_h(LN(h) . b1^T) (the score GEMM folds the LayerNorm
    from the producer's partials st and applies the 80-column softmax in its epilogue), h = P . b2^T + b_o + h
    (writing st_out, the next LayerNorm's partials).  Image g of h (rows_per_img rows each, a multiple of 256) uses
    prompt row s0 + (g % mod if mod else g).  P: [M, KP] buffer whose columns past H*80 are zero."""
    HP, KP, C = m.HP, m.KP, m.C
    gemm(h, m.b1[s0:], out=P, N=HP, K=C, ldw=C, ldc=KP, ln_in=st, ln_c=m.c[s0:], bias=m.d[s0:], act="softmax",
         sm_len=Lk, bsel=(rows_per_img, mod, HP * C, HP))
    gemm(P, m.b2[s0:], N=C, K=KP, ldw=KP, bias=bias_o, residual=h, out=h, ln_out=st_out,
         bsel=(rows_per_img, mod, C * KP, 0))
    return h


def xattn_consts(b1, rows, K, kv, ldkv, kv_rstride, dq, heads, slot, Lk, scale, c, d):
    """LayerNorm-fold constants of the cross-attention score matrix rows (fd_xattn_consts): c = rowsum(b1 rows),
    d = scale * K_j,h . dq_h (0 for pad keys)."""
    L.check(L.load().fd_xattn_consts(L.ptr(b1), b1.stride(-2), rows, K, L.ptr(kv), ldkv, kv_rstride, L.ptr(dq), heads,
                                     slot, Lk, scale, L.ptr(c), L.ptr(d), L.dtype_code(b1.dtype), L.stream()),
            "fd_xattn_consts")


def pack_e4m3(w):
    """Weights -> OCP e4m3 bytes [N][K] (uint8) exactly as utils/system.py:20 (``.to(torch.float8_e4m3fn)``:
    unscaled, RNE, no saturation), for gemm_e4m3(w_scale=1)."""
    return w.to(torch.float8_e4m3fn).view(torch.uint8).contiguous()


def quant_rows_e4m3(x, q=None, scale=None, M=None, K=None, ldx=None):
    """x [M, K] bf16/f16 -> (q uint8 [M, K] e4m3, scale fp32 [M]) with x ~= q * scale per row."""
    K = x.shape[-1] if K is None else K
    M = x.numel() // x.shape[-1] if M is None else M
    ldx = x.stride(-2) if ldx is None else ldx
    if q is None:
        q = torch.empty((M, K), dtype=torch.uint8, device=x.device)
    if scale is None:
        scale = torch.empty((M,), dtype=torch.float32, device=x.device)
    L.check(L.load().fd_quant_rows_e4m3(L.ptr(x), ldx, L.ptr(q), q.stride(0), L.ptr(scale), M, K,
                                        L.dtype_code(x.dtype), L.stream()), "fd_quant_rows_e4m3")
    return q, scale


def layer_norm_e4m3(x, gamma, beta, eps=1e-5, q=None, scale=None):
    """LayerNorm(x) quantized per row to e4m3 in one launch: (q uint8 [M, C], scale fp32 [M]) bitwise equal to
    quant_rows_e4m3(layer_norm(x))."""
    M, C = x.shape
    if q is None:
        q = torch.empty((M, C), dtype=torch.uint8, device=x.device)
    if scale is None:
        scale = torch.empty((M,), dtype=torch.float32, device=x.device)
    L.check(L.load().fd_layer_norm_e4m3(L.ptr(x), x.stride(0), L.ptr(q), q.stride(0), L.ptr(scale), L.ptr(gamma),
                                        L.ptr(beta), M, C, eps, L.dtype_code(x.dtype), L.stream()),
            "fd_layer_norm_e4m3")
    return q, scale


def gemm_e4m3(a8, a_scale, w8, out=None, bias=None, residual=None, w_scale=1.0, act="none", out_dtype=torch.bfloat16):
    """out[M, N (N/2 for geglu)] = act(a_scale[m] * w_scale * (a8[M, K] @ w8[N, K]^T) + bias) + residual on the
    fp8 MFMA (geglu: w8 / bias packed by pack_geglu)."""
    M, K = a8.shape
    N = w8.shape[0]
    if w8.shape[1] != K:
        raise ValueError(f"gemm_e4m3: K mismatch {a8.shape} x {w8.shape}")
    nout = N // 2 if act == "geglu" else N
    if out is None:
        out = torch.empty((M, nout), dtype=out_dtype, device=a8.device)
    if residual is not None and residual.dtype != out.dtype:
        raise ValueError(f"gemm_e4m3: residual dtype {residual.dtype} != output dtype {out.dtype}")
    args = (L.ptr(a8), a8.stride(0), L.ptr(a_scale), L.ptr(w8), w8.stride(0), w_scale, L.ptr(out), out.stride(0),
            M, N, K, L.ptr(bias), L.ptr(residual), 0 if residual is None else residual.stride(0), L.ACT[act],
            L.dtype_code(out.dtype), L.stream())
    _timed("gemm_e4m3", 2.0 * M * N * K, 0.0, lambda: L.check(L.load().fd_gemm_e4m3(*args), "fd_gemm_e4m3"))
    return out


class MX:
    """An OCP MX e4m3 activation: q uint8 [M, K] (e4m3 bytes) and s uint8 [M, K/32] (E8M0 block scales, byte =
    exponent + 127), the format the use_fp8 model's producers (flash attention, GEGLU, LayerNorm) write for
    fd_gemm_mxe4m3.  ``s`` rows are padded to a multiple of 4 bytes (the GEMM reads one dword per 128 elements)."""

    def __init__(self, M, K, device, q=None, s=None):
        if K % 32:
            raise ValueError(f"MX: K={K} not a multiple of 32")
        self.q = torch.empty((M, K), dtype=torch.uint8, device=device) if q is None else q
        self.s = torch.empty((M, -(-K // 128) * 4), dtype=torch.uint8, device=device) if s is None else s

    @property
    def shape(self):
        return tuple(self.q.shape)

    def dequant(self):
        """fp32 values (host-side checking only)."""
        M, K = self.q.shape
        e = self.s[:, :K // 32].to(torch.float32) - 127.0
        return self.q.view(torch.float8_e4m3fn).float() * torch.exp2(e).repeat_interleave(32, dim=1)


def _mx_out_tiles(M, nout, geglu):
    """Whether fd_gemm_mxe4m3 has a tile shape for an MX output (its plan_e4m3 with mx_out): (rows, output columns)
    dividing (M, nout) with the columns a multiple of 32."""
    tiles = [(256, 64)] if geglu else [(256, 160), (256, 128), (128, 160), (64, 160)]
    return any(M % bm == 0 and nout % bn == 0 for bm, bn in tiles)


def quant_rows_mx(x, out=None):
    """x [M, K] (bf16 / f16 / f32, K % 32 == 0) -> MX (fd_quant_rows_mx)."""
    M, K = x.shape
    out = MX(M, K, x.device) if out is None else out
    L.check(L.load().fd_quant_rows_mx(L.ptr(x), x.stride(0), L.ptr(out.q), out.q.stride(0), L.ptr(out.s),
                                      out.s.stride(0), M, K, L.dtype_code(x.dtype), L.stream()), "fd_quant_rows_mx")
    return out


def layer_norm_mx(x, gamma, beta, eps=1e-5, out=None):
    """LayerNorm(x) rounded to x.dtype and written as MX (bitwise quant_rows_mx(layer_norm(x)))."""
    M, C = x.shape
    out = MX(M, C, x.device) if out is None else out
    L.check(L.load().fd_layer_norm_mx(L.ptr(x), x.stride(0), L.ptr(out.q), out.q.stride(0), L.ptr(out.s),
                                      out.s.stride(0), L.ptr(gamma), L.ptr(beta), M, C, eps, L.dtype_code(x.dtype),
                                      L.stream()), "fd_layer_norm_mx")
    return out


def gemm_mx(a, w8, out=None, bias=None, residual=None, w_scale=1.0, act="none", out_dtype=torch.bfloat16):
    """out = act(w_scale * (dequant(a) @ w8^T) + bias) + residual on the block-scaled e4m3 MFMA (fd_gemm_mxe4m3);
    a: MX [M, K]; w8 e4m3 bytes [N, K] (geglu: packed by pack_geglu, N/2 output columns).  out_dtype "mx" (or an
    MX ``out``): the output is written as MX e4m3 (GEGLU producer of the ff-out GEMM)."""
    M, K = a.q.shape
    N = w8.shape[0]
    if w8.shape[1] != K:
        raise ValueError(f"gemm_mx: K mismatch {a.q.shape} x {w8.shape}")
    nout = N // 2 if act == "geglu" else N
    mx_out = isinstance(out, MX) or out_dtype == "mx"
    if out is None:
        out = MX(M, nout, a.q.device) if mx_out else torch.empty((M, nout), dtype=out_dtype, device=a.q.device)
    if mx_out and residual is not None:
        raise ValueError("gemm_mx: an MX output takes no residual (the C entry point rejects it too)")
    if mx_out and not _mx_out_tiles(M, nout, act == "geglu"):
        # no tile shape covers this output with whole 32-column blocks (small test sizes): the fp32 output, then
        # fd_quant_rows_mx -- the same bytes the fused epilogue writes (it quantizes the same fp32 values)
        y = gemm_mx(a, w8, bias=bias, w_scale=w_scale, act=act, out_dtype=torch.float32)
        return quant_rows_mx(y, out=out)
    if mx_out:
        cq, cs, ldcs, code = out.q, out.s, out.s.stride(0), 3
    else:
        cq, cs, ldcs, code = out, None, 0, L.dtype_code(out.dtype)
        if residual is not None and residual.dtype != out.dtype:
            raise ValueError(f"gemm_mx: residual dtype {residual.dtype} != output dtype {out.dtype}")
    args = (L.ptr(a.q), a.q.stride(0), L.ptr(a.s), a.s.stride(0), L.ptr(w8), w8.stride(0), w_scale, L.ptr(cq),
            cq.stride(0), L.ptr(cs), ldcs, M, N, K, L.ptr(bias), L.ptr(residual),
            0 if residual is None else residual.stride(0), L.ACT[act], code, L.stream())
    _timed("gemm_e4m3", 2.0 * M * N * K, 0.0, lambda: L.check(L.load().fd_gemm_mxe4m3(*args), "fd_gemm_mxe4m3"))
    return out


def flash_attn_mx(q, k, v, out, batch, heads, Lq, Lk, ldq, ldk, ldv, qbs, kbs, vbs, kv_mod=0, scale=0.125):
    """flash_attn with the output written as MX (out: MX [batch * Lq, heads * 64]); the row of (b, q) is b * Lq + q."""
    ldo = out.q.stride(0)
    lds = out.s.stride(0)
    _timed("flash_attn", 4.0 * batch * heads * Lq * Lk * 64, 0, label=f"flash b={batch} h={heads} Lq={Lq} Lk={Lk}",
           launch=lambda: L.check(
        L.load().fd_flash_attn_mx(L.ptr(q), ldq, qbs, L.ptr(k), ldk, kbs, L.ptr(v), ldv, vbs, L.ptr(out.q), ldo,
                                  Lq * ldo, L.ptr(out.s), lds, Lq * lds, batch, heads, Lq, Lk, kv_mod, 0, scale,
                                  L.dtype_code(q.dtype), L.stream()), "fd_flash_attn_mx"))
    return out


def linear_e4m3(x, w8, bias=None, residual=None, act="none", out=None):
    """nn.Linear of a quantize_8bit UNet on the fp8 MFMA: per-row e4m3 activations x e4m3 weight bytes."""
    q, s = quant_rows_e4m3(x)
    return gemm_e4m3(q, s, w8, out=out, bias=bias, residual=residual, act=act, out_dtype=x.dtype)


def fold_layer_norm(w, gamma, beta, bias=None, dtype=torch.bfloat16):
    """LayerNorm(x; gamma, beta) @ w^T + bias == rstd * (x @ w'^T - mean * c) + d  with
    w' = w * gamma (per input column, rounded to the GEMM dtype), c = rowsum(w') of the rounded values and
    d = w @ beta + bias (fp64).  Returns (w', c, d) for gemm(..., ln_in=..., ln_c=c, bias=d)."""
    w64 = w.double()
    wp = (w64 * gamma.double()[None, :]).to(dtype)
    c = wp.double().sum(1).float()
    d = w64 @ beta.double()
    if bias is not None:
        d = d + bias.double()
    return wp.contiguous(), c.contiguous(), d.float().contiguous()


def _conv_params(x, wp, bias, nimg, H, W, stride, pad, upsample, x2, C1, out, rowbias, residual, act, out_dtype,
                 upsample_size, lda, alpha):
    Cout, K = wp.shape
    Cin = K // 9
    Hl, Wl = ((2 * H, 2 * W) if upsample_size is None else tuple(upsample_size)) if upsample else (H, W)
    Hout = (Hl + 2 * pad - 3) // stride + 1
    Wout = (Wl + 2 * pad - 3) // stride + 1
    if stride == 2 and pad == 0:  # VAE Downsample2D: F.pad (0,1,0,1) then conv(k3, s2, p0)
        Hout, Wout = Hl // 2, Wl // 2
    M = nimg * Hout * Wout
    odt = out_dtype or x.dtype
    if out is None:
        out = torch.empty((M, Cout), dtype=odt, device=x.device)
    p = L.GemmParams()
    p.A, p.B, p.C = x.data_ptr(), wp.data_ptr(), out.data_ptr()
    p.C1 = 0 if x2 is None else C1
    p.lda = (Cin if lda is None else lda) if x2 is None else C1
    p.ldb, p.ldc = K, out.stride(-2)
    p.M, p.N, p.K, p.batch = M, Cout, K, 1
    p.bias = bias.data_ptr() if bias is not None else None
    if residual is not None:
        p.residual, p.ldr = residual.data_ptr(), residual.stride(-2)
        p.residual_rows = _rows(residual, p.ldr, Cout)
    if rowbias is not None:
        p.rowbias, p.rowbias_ld, p.rows_per_group = rowbias.data_ptr(), rowbias.stride(0), Hout * Wout
        p.rowbias_rows = _rows(rowbias, p.rowbias_ld, Cout)
    else:
        p.rows_per_group = 1
    p.alpha, p.act = alpha, L.ACT[act]
    p.dtype, p.out_dtype = L.dtype_code(x.dtype), L.dtype_code(odt)
    p.conv, p.nimg, p.Hin, p.Win, p.Cin = 1, nimg, H, W, Cin
    p.Hout, p.Wout, p.stride, p.pad, p.upsample = Hout, Wout, stride, pad, int(upsample)
    p.A2 = x2.data_ptr() if x2 is not None else None
    groups = _TILE_GROUPS[-1]
    p.m_ref = p.M // groups if groups > 1 and p.M % groups == 0 else p.M
    return p, out


def conv3x3(x, wp, bias, nimg, H, W, stride=1, pad=1, upsample=False, x2=None, C1=None, out=None, rowbias=None,
            residual=None, act="none", out_dtype=None, upsample_size=None, gn=None, lda=None, alpha=1.0, gn_in=None):
    """Implicit-GEMM 3x3 conv on NHWC x [nimg*H*W, Cin] (or concat(x, x2) along C) with packed weight wp.
    upsample=True: nearest-resize to upsample_size (default 2H x 2W) folded into the gather.  lda: pixel stride
    of x when it is a channel slice of a wider buffer (default Cin); alpha scales the accumulator (before bias).
    gn_in = (affine, silu): the consumer GroupNorm (+ SiLU) of x applied in the conv's staging pass
    (fd_gemm_params.gi_affine; affine from group_norm_affine) -- only where halo_conv_rows() says the halo-staged
    kernel takes this conv."""
    p, out = _conv_params(x, wp, bias, nimg, H, W, stride, pad, upsample, x2, C1, out, rowbias, residual, act,
                          out_dtype, upsample_size, lda, alpha)
    if gn_in is not None:
        p.gi_affine, p.gi_silu = gn_in[0].data_ptr(), int(gn_in[1])
    if gn is not None:
        gn.attach(p)
    _attach_ws(p, x.device)
    _launch_gemm(p, "fd_gemm(conv)")
    if gn is not None:
        gn.collect(p)
    return out


class _WShape:  # a [Cout, 9 Cin] stand-in for _conv_params (the phase weights are [4 Cout, 4 Cin])
    def __init__(self, w, cout, cin):
        self.shape, self._p = (cout, 9 * cin), w.data_ptr()

    def data_ptr(self):
        return self._p


def conv3x3_up2_params(x, wph, bias, nimg, H, W, out=None, residual=None, act="none", gn=None):
    Cout, Cin = wph.shape[0] // 4, wph.shape[1] // 4
    p, out = _conv_params(x, _WShape(wph, Cout, Cin), bias, nimg, H, W, 1, 1, True, None, None, out, None, residual,
                          act, None, None, None, 1.0)
    p.K, p.ldb, p.up_phase = 4 * Cin, wph.stride(0), 1
    return p, out


def conv3x3_up2(x, wph, bias, nimg, H, W, out=None, residual=None, act="none", gn=None):
    """Upsample2D (nearest x2 + 3x3 conv) on NHWC x [nimg*H*W, Cin] in four 2x2 phases with the
    pack_conv3x3_up2 weights wph [4*Cout, 4*Cin] -> [nimg*2H*2W, Cout] (fd_gemm_params.up_phase; the halo-staged
    kernel; up2_phase_ok() says whether it takes the shape)."""
    p, out = conv3x3_up2_params(x, wph, bias, nimg, H, W, out, residual, act)
    if gn is not None:
        gn.attach(p)
    _attach_ws(p, x.device)
    _launch_gemm(p, "fd_gemm(conv up2 phases)")
    if gn is not None:
        gn.collect(p)
    return out


def up2_phase_ok(x, wph, nimg, H, W):
    """True when fd_gemm runs this x2 upsample conv in the phase form (shapes only)."""
    dummy = torch.empty((1, wph.shape[0] // 4), dtype=x.dtype, device=x.device)
    p, _ = conv3x3_up2_params(x, wph, None, nimg, H, W, out=dummy)
    p.C, p.ldc = x.data_ptr(), wph.shape[0] // 4
    p.M = nimg * 4 * H * W
    return int(L.load().fd_conv_halo_plan(ctypes.byref(p))) > 0


def gn_conv3x3(x, gamma, beta, wp, bias, nimg, H, W, eps, silu=True, groups=32, stats=None, **kw):
    """conv3x3(GroupNorm(+SiLU)(x)) -- the norm -> SiLU -> conv of a ResnetBlock2D.  Where the halo-staged conv
    takes the conv, the GroupNorm is its per-(image, channel) affine applied in the conv's staging pass (no
    normalised tensor is written or read); else a GroupNorm pass, then the conv.  stats: GnStats of x from its
    producer's epilogue (skips the statistics pass either way)."""
    C = x.shape[-1]
    # the in-staging transform costs ~1.2-1.5 us per 64-channel chunk, a GroupNorm apply pass ~10-14 us at the UNet's
    # sizes: folding pays up to ~10 chunks (probes/conv_ab.py, profiles/r04d_conv_ab.jsonl, r04e_conv_ab.jsonl);
    # wider inputs take the apply pass and the plain halo conv
    if C <= knobs.get("FD_HALO_GN_CIN_MAX") and halo_conv_rows(
            x, wp, nimg, H, W, upsample=kw.get("upsample", False), upsample_size=kw.get("upsample_size"),
            residual=kw.get("residual"), rowbias=kw.get("rowbias"), out=kw.get("out"),
            out_dtype=kw.get("out_dtype")) > 0:
        aff = group_norm_affine(x, gamma, beta, nimg, H * W, C, groups, eps, stats=stats)
        return conv3x3(x, wp, bias, nimg, H, W, gn_in=(aff, silu), **kw)
    h = group_norm(x, gamma, beta, nimg, H * W, C, groups, eps, silu=silu, stats=stats)
    return conv3x3(h, wp, bias, nimg, H, W, **kw)


def halo_conv_rows(x, wp, nimg, H, W, stride=1, pad=1, upsample=False, x2=None, upsample_size=None, lda=None,
                   residual=None, rowbias=None, out=None, out_dtype=None):
    """Rows per GroupNorm-statistics block the halo-staged conv kernel would write for this conv (256 / 128), 0 when
    fd_gemm takes it on the implicit GEMM (then a consumer GroupNorm must run as its own pass).  Shapes only; the
    residual / row bias / output the real call passes (their pointers and pitches) enter the plan's alignment rules."""
    dummy = torch.empty((1, wp.shape[0]), dtype=out_dtype or x.dtype, device=x.device)
    p, _ = _conv_params(x, wp, None, nimg, H, W, stride, pad, upsample, x2, None if x2 is None else 0, dummy, rowbias,
                        residual, "none", out_dtype, upsample_size, lda, 1.0)
    if out is not None:
        p.C, p.ldc = out.data_ptr(), out.stride(-2)
    else:
        p.C, p.ldc = x.data_ptr(), wp.shape[0]  # alignment / stride stand-ins for a fresh output allocation
    return int(L.load().fd_conv_halo_plan(ctypes.byref(p)))


def halo_conv_pt(x, wp, nimg, H, W, upsample=False, upsample_size=None, residual=False, rowbias=False, gn_in=False):
    """Workgroups of the halo kernel's persistent form for this conv (0: one workgroup per tile, or not the halo
    kernel).  Shapes only (gn_in: with a consumer GroupNorm folded into the staging)."""
    dummy = torch.empty((1, wp.shape[0]), dtype=x.dtype, device=x.device)
    p, _ = _conv_params(x, wp, None, nimg, H, W, 1, 1, upsample, None, None, dummy, None, None, "none", None,
                        upsample_size, None, 1.0)
    p.C, p.ldc = x.data_ptr(), wp.shape[0]
    if gn_in:
        p.gi_affine = x.data_ptr()
    if residual:
        p.residual, p.ldr, p.residual_rows = x.data_ptr(), wp.shape[0], p.M
    if rowbias:
        p.rowbias, p.rowbias_ld, p.rowbias_rows = x.data_ptr(), wp.shape[0], nimg
    return int(L.load().fd_conv_halo_pt(ctypes.byref(p)))


def conv3x3_narrow(x, w32, bias, nimg, H, W, out_dtype=None, out=None, gn_in=None):
    """3x3 conv (stride 1, pad 1) with Cout <= 4 on NHWC x [nimg*H*W, Cin]: w32 fp32 [Cout, 9*Cin] (tap-major, the
    pack_conv3x3 layout).  The VAE decoder's conv_out.  gn_in = (affine, silu): the GroupNorm (+ SiLU) in front of
    it applied to the staged input (affine from group_norm_affine; fd_conv3x3_narrow_gn)."""
    Cout, K = w32.shape
    Cin = K // 9
    odt = out_dtype or x.dtype
    if out is None:
        out = torch.empty((nimg * H * W, Cout), dtype=odt, device=x.device)
    if gn_in is None:
        fn = lambda: L.check(L.load().fd_conv3x3_narrow(L.ptr(x), L.ptr(w32), L.ptr(bias), L.ptr(out), nimg, H, W, Cin,
                                                        Cout, L.dtype_code(x.dtype), L.dtype_code(odt), L.stream()),
                             "fd_conv3x3_narrow")
    else:
        aff, silu = gn_in
        fn = lambda: L.check(L.load().fd_conv3x3_narrow_gn(L.ptr(x), L.ptr(w32), L.ptr(bias), L.ptr(aff), int(silu),
                                                           L.ptr(out), nimg, H, W, Cin, Cout, L.dtype_code(x.dtype),
                                                           L.dtype_code(odt), L.stream()), "fd_conv3x3_narrow_gn")
    _timed("conv_narrow", 2.0 * nimg * H * W * Cout * K, 0.0, label=f"conv3x3_narrow M={nimg * H * W} N={Cout} K={K}",
           launch=fn)
    return out


def conv_direct(x, w, bias, nimg, H, W, Cin, ksize=3, stride=1, pad=1, in_scale=1.0, out_dtype=None, out=None):
    """Direct conv for Cin < 64: x NHWC, w fp32 [Cout, k, k, Cin]."""
    Cout = w.shape[0]
    Hout, Wout = (H + 2 * pad - ksize) // stride + 1, (W + 2 * pad - ksize) // stride + 1
    odt = out_dtype or x.dtype
    if out is None:
        out = torch.empty((nimg * Hout * Wout, Cout), dtype=odt, device=x.device)
    L.check(L.load().fd_conv2d_direct(L.ptr(x), L.ptr(w), L.ptr(bias), L.ptr(out), nimg, H, W, Cin, Cout, ksize,
                                      stride, pad, in_scale, L.dtype_code(x.dtype), L.dtype_code(odt), L.stream()),
            "fd_conv2d_direct")
    return out


# --------------------------------------------------------------------------------------- norms
def group_norm(x, gamma, beta, nimg, HW, C, groups=32, eps=1e-5, silu=False, out=None, stats=None):
    """GroupNorm (+SiLU) of NHWC x.  stats: a GnStats the producer of x filled (gn=...): the statistics pass is
    skipped (fd_group_norm_partials)."""
    if out is None:
        out = torch.empty_like(x)
    if stats is not None and stats.done:
        if (stats.nimg, stats.HW, stats.groups) != (nimg, HW, groups):
            raise ValueError("group_norm: stats were gathered for a different shape")
        st = _gn_ws(nimg * groups * 8, x.device)
        _timed("group_norm", 0, 2.0 * nimg * HW * C * x.element_size(), lambda: L.check(
            L.load().fd_group_norm_partials(L.ptr(x), L.ptr(out), L.ptr(gamma), L.ptr(beta), nimg, HW, C, groups, eps,
                                            int(silu), L.ptr(stats.part), stats.rows, L.ptr(st), L.dtype_code(x.dtype),
                                            L.stream()), "fd_group_norm_partials"))
        return out
    nb = L.load().fd_group_norm_ws_bytes(nimg, HW, C, groups)
    ws = _gn_ws(nb, x.device)
    _timed("group_norm", 0, 2.0 * nimg * HW * C * x.element_size(), lambda: L.check(
        L.load().fd_group_norm(L.ptr(x), L.ptr(out), L.ptr(gamma), L.ptr(beta), nimg, HW, C, groups, eps, int(silu),
                               L.dtype_code(x.dtype), L.ptr(ws), L.stream()), "fd_group_norm"))
    return out


def group_norm_affine(x, gamma, beta, nimg, HW, C, groups=32, eps=1e-5, stats=None):
    """The GroupNorm of NHWC x as a per-(image, channel) fp32 affine [nimg * C + 64, 2] (scale, shift) for a consumer
    that applies it itself (conv3x3(..., gn_in=(affine, silu))).  stats: a GnStats the producer of x filled (no
    statistics pass)."""
    aff = torch.empty((nimg * C + 64, 2), dtype=torch.float32, device=x.device)
    if stats is not None and stats.done:
        if (stats.nimg, stats.HW, stats.groups) != (nimg, HW, groups):
            raise ValueError("group_norm_affine: stats were gathered for a different shape")
        ws = _gn_ws(nimg * groups * 8, x.device)
        part, rows = L.ptr(stats.part), stats.rows
    else:
        ws = _gn_ws(L.load().fd_group_norm_ws_bytes(nimg, HW, C, groups), x.device)
        part, rows = None, 0
    _timed("group_norm", 0, 1.0 * nimg * HW * C * x.element_size() * (0 if part else 1), lambda: L.check(
        L.load().fd_group_norm_affine(L.ptr(x), part, rows, L.ptr(gamma), L.ptr(beta), nimg, HW, C, groups, eps,
                                      L.ptr(ws), L.ptr(aff), L.dtype_code(x.dtype), L.stream()),
        "fd_group_norm_affine"))
    return aff


def layer_norm(x, gamma, beta, eps=1e-5, out=None, M=None, ldx=None):
    C = gamma.shape[0]
    M = x.numel() // x.shape[-1] if M is None else M
    if out is None:
        out = torch.empty((M, C), dtype=x.dtype, device=x.device)
    _timed("layer_norm", 0, 2.0 * M * C * x.element_size(), lambda: L.check(
        L.load().fd_layer_norm(L.ptr(x), x.stride(-2) if ldx is None else ldx, L.ptr(out), out.stride(-2),
                               L.ptr(gamma), L.ptr(beta), M, C, eps, L.dtype_code(x.dtype), L.stream()),
        "fd_layer_norm"))
    return out


# --------------------------------------------------------------------------------------- attention
def flash_attn(q, k, v, out, batch, heads, Lq, Lk, ldq, ldk, ldv, ldo, qbs, kbs, vbs, obs, kv_mod=0, scale=0.125,
               causal=False):
    _timed("flash_attn", 4.0 * batch * heads * Lq * Lk * 64, 0, label=f"flash b={batch} h={heads} Lq={Lq} Lk={Lk}",
           launch=lambda: L.check(
        L.load().fd_flash_attn(L.ptr(q), ldq, qbs, L.ptr(k), ldk, kbs, L.ptr(v), ldv, vbs, L.ptr(out), ldo, obs,
                               batch, heads, Lq, Lk, kv_mod, int(causal), scale, L.dtype_code(q.dtype), L.stream()),
        "fd_flash_attn"))
    return out


def flash_attn_d512(qkv, out, nimg, T, scale=512 ** -0.5, split=None):
    """Single-head d=512 attention on the qkv projection [nimg*T, 1536] (q | k | v) -> out [nimg*T, 512].
    split (default: the FD_D512_SPLIT path switch): the 8-wave kernel with the keys split over
    fd_flash_attn_d512_ksplit(nimg, T) workgroups per 128-query block, merged by a second launch through an fp32
    scratch of nimg * ks * T * 513 floats; else the 4-wave single-pass kernel."""
    from . import knobs
    ld = qkv.stride(0)
    if split is None:
        split = knobs.get("FD_D512_SPLIT") != 0
    if split:
        lib = L.load()
        ks = lib.fd_flash_attn_d512_ksplit(nimg, T)
        nfl = nimg * ks * T * 513 if ks > 1 else 0
        part = torch.empty(max(nfl, 4), dtype=torch.float32, device=qkv.device)
        _timed("flash_attn_d512", 4.0 * nimg * T * T * 512, 0, label=f"flash512 n={nimg} T={T} ks={ks}",
               launch=lambda: L.check(lib.fd_flash_attn_d512_split(
                   L.ptr(qkv), L.ptr(qkv[:, 512:]), L.ptr(qkv[:, 1024:]), ld, T * ld, L.ptr(out), out.stride(0),
                   T * out.stride(0), nimg, T, scale, L.dtype_code(qkv.dtype), L.ptr(part), nfl, ks, L.stream()),
                   "fd_flash_attn_d512_split"))
        return out
    _timed("flash_attn_d512", 4.0 * nimg * T * T * 512, 0, label=f"flash512 n={nimg} T={T}", launch=lambda: L.check(
        L.load().fd_flash_attn_d512(L.ptr(qkv), L.ptr(qkv[:, 512:]), L.ptr(qkv[:, 1024:]), ld, T * ld, L.ptr(out),
                                    out.stride(0), T * out.stride(0), nimg, T, scale, L.dtype_code(qkv.dtype),
                                    L.stream()), "fd_flash_attn_d512"))
    return out


def embed_tokens(ids, tok, pos, out, batch, L_):
    """ids int32 [batch*L_] (device); tok [vocab, D], pos [>=L_, D] -> out [batch*L_, D]."""
    D = tok.shape[1]
    L.check(L.load().fd_embed_tokens(L.ptr(ids), L.ptr(tok), L.ptr(pos), L.ptr(out), batch, L_, D, tok.shape[0],
                                     L.dtype_code(tok.dtype), L.stream()), "fd_embed_tokens")
    return out


def mha_seq_axis(qkv, out, L_, groups, N, E, heads):
    L.check(L.load().fd_mha_seq_axis(L.ptr(qkv), L.ptr(out), L_, groups, N, E, heads, L.dtype_code(qkv.dtype),
                                     L.stream()), "fd_mha_seq_axis")
    return out


def softmax_rows(s, out, R, C, scale, ldp=None):
    L.check(L.load().fd_softmax_rows(L.ptr(s), L.ptr(out), R, C, C if ldp is None else ldp, scale,
                                     L.dtype_code(out.dtype), L.stream()),
            "fd_softmax_rows")
    return out


# --------------------------------------------------------------------------------------- elementwise
def concat_channels(a, C1, b, C2, out, M, gn=None):
    """out = concat(a [M, C1], b [M, C2]) along channels.  gn: a GnStats for out's GroupNorm consumer -- the concat
    then also writes fd_group_norm's own statistics partials (fd_concat_channels_gn, one launch instead of the concat
    and the statistics pass; same bits); gn.done stays False where the shape does not allow it (HW not a multiple of
    the chunk rows)."""
    if gn is not None:
        gn.done, gn.rows = False, 0
        rows = int(L.load().fd_group_norm_chunk_rows(gn.nimg, gn.HW))
        C = C1 + C2
        if (rows > 0 and gn.HW % rows == 0 and gn.nimg * gn.HW == M and C % gn.groups == 0
                and (C // 8 <= 256 or C % 16 == 0)):
            need = gn.nimg * (gn.HW // rows) * gn.groups * 2
            if gn.part.numel() < need:
                gn.part = torch.empty((need,), dtype=torch.float32, device=out.device)
            L.check(L.load().fd_concat_channels_gn(L.ptr(a), C1, L.ptr(b), C2, L.ptr(out), gn.nimg, gn.HW, gn.groups,
                                                   L.ptr(gn.part), L.dtype_code(a.dtype), L.stream()),
                    "fd_concat_channels_gn")
            gn.done, gn.rows = True, rows
            return out
    L.check(L.load().fd_concat_channels(L.ptr(a), C1, L.ptr(b), C2, L.ptr(out), M, L.dtype_code(a.dtype), L.stream()),
            "fd_concat_channels")
    return out


def unary(x, out, act="none"):
    L.check(L.load().fd_unary(L.ptr(x), L.ptr(out), x.numel(), L.ACT[act], L.dtype_code(x.dtype),
                              L.dtype_code(out.dtype), L.stream()), "fd_unary")
    return out


def add_strided(x, ldx, a, lda, out, ldy, M, N):
    L.check(L.load().fd_add_strided(L.ptr(x), ldx, L.ptr(a), lda, L.ptr(out), ldy, M, N, L.dtype_code(x.dtype),
                                    L.dtype_code(out.dtype), L.stream()), "fd_add_strided")
    return out


def axpby(x, z, out, alpha, beta, M=None, N=None):
    """out = alpha * x + beta * z over [M, N] with each tensor's own row stride (out may alias z)."""
    M = x.shape[0] if M is None else M
    N = x.shape[-1] if N is None else N
    L.check(L.load().fd_axpby(L.ptr(x), x.stride(0), L.ptr(z), z.stride(0), L.ptr(out), out.stride(0), M, N,
                              float(alpha), float(beta), L.dtype_code(x.dtype), L.stream()), "fd_axpby")
    return out


def nchw_to_nhwc(x, out, nimg, C, HW, scale=1.0):
    L.check(L.load().fd_nchw_to_nhwc(L.ptr(x), L.ptr(out), nimg, C, HW, scale, L.dtype_code(x.dtype),
                                     L.dtype_code(out.dtype), L.stream()), "fd_nchw_to_nhwc")
    return out


def nhwc_to_nchw(x, out, nimg, C, HW, scale=1.0):
    L.check(L.load().fd_nhwc_to_nchw(L.ptr(x), L.ptr(out), nimg, C, HW, scale, L.dtype_code(x.dtype),
                                     L.dtype_code(out.dtype), L.stream()), "fd_nhwc_to_nchw")
    return out


def transpose(x, ldx, out, ldy, R, C, batch=1, sx=0, sy=0):
    L.check(L.load().fd_transpose(L.ptr(x), ldx, L.ptr(out), ldy, R, C, batch, sx, sy, L.dtype_code(x.dtype),
                                  L.stream()), "fd_transpose")
    return out


def time_features(t, time_ids, text_embeds, tfeat, afeat, batch):
    L.check(L.load().fd_time_features(L.ptr(t), L.ptr(time_ids), L.ptr(text_embeds), L.ptr(tfeat), L.ptr(afeat), batch,
                                      L.dtype_code(tfeat.dtype), L.stream()), "fd_time_features")


# --------------------------------------------------------------------------------------- denoise loop
def euler_scale_divisor(sigma):
    """(sigma^2 + 1)^0.5 in fp32 exactly as torch computes scale_model_input's divisor from the fp32 sigmas."""
    sg = torch.tensor(float(sigma), dtype=torch.float32)
    return float((sg ** 2 + 1) ** 0.5)


def tlc_scale_input(canvas, row_org, col_org, H, W, kh, kw, tile_begin, ntiles, cfg, sigma, out, t_out=None,
                    timestep=None):
    """Tiles of the canvas / (sigma^2 + 1)^0.5 (correctly rounded fp32 division), CFG-duplicated, NHWC.  t_out (fp32,
    contiguous): also filled with ``timestep`` by the same launch (fd_tlc_scale_input_t)."""
    if t_out is None:
        L.check(L.load().fd_tlc_scale_input(L.ptr(canvas), L.ptr(row_org), row_org.numel(), L.ptr(col_org),
                                            col_org.numel(), H, W, kh, kw, tile_begin, ntiles, cfg,
                                            euler_scale_divisor(sigma), L.ptr(out),
                                            L.dtype_code(out.dtype), L.stream()), "fd_tlc_scale_input")
        return out
    if t_out.dtype != torch.float32 or not t_out.is_contiguous():
        raise ValueError("tlc_scale_input: t_out must be a contiguous fp32 tensor")
    L.check(L.load().fd_tlc_scale_input_t(L.ptr(canvas), L.ptr(row_org), row_org.numel(), L.ptr(col_org),
                                          col_org.numel(), H, W, kh, kw, tile_begin, ntiles, cfg,
                                          euler_scale_divisor(sigma), L.ptr(out), L.dtype_code(out.dtype),
                                          L.ptr(t_out), t_out.numel(), float(timestep), L.stream()),
            "fd_tlc_scale_input_t")
    return out


def tlc_cfg_euler_step(eps, canvas, row_org, col_org, H, W, kh, kw, tile_begin, ntiles, cfg, guidance, rescale, sigma,
                       sigma_next, out_tiles):
    L.check(L.load().fd_tlc_cfg_euler_step(L.ptr(eps), L.ptr(canvas), L.ptr(row_org), row_org.numel(), L.ptr(col_org),
                                           col_org.numel(), H, W, kh, kw, tile_begin, ntiles, cfg, guidance, rescale,
                                           sigma, sigma_next, L.ptr(out_tiles), L.dtype_code(eps.dtype), L.stream()),
            "fd_tlc_cfg_euler_step")
    return out_tiles


def tlc_blend(tiles, weights, row_org, col_org, C, H, W, kh, kw, canvas):
    L.check(L.load().fd_tlc_blend(L.ptr(tiles), L.ptr(weights), L.ptr(row_org), row_org.numel(), L.ptr(col_org),
                                  col_org.numel(), C, H, W, kh, kw, L.ptr(canvas), L.stream()), "fd_tlc_blend")
    return canvas


def tlc_grids_nhwc(canvas, row_org, col_org, H, W, C, kh, kw, tile_begin, ntiles, cfg, out):
    L.check(L.load().fd_tlc_grids_nhwc(L.ptr(canvas), L.ptr(row_org), row_org.numel(), L.ptr(col_org), col_org.numel(),
                                       H, W, C, kh, kw, tile_begin, ntiles, cfg, L.ptr(out), L.dtype_code(canvas.dtype),
                                       L.stream()), "fd_tlc_grids_nhwc")
    return out


def vae_sample_add_noise(moments, post_eps, noise, out, HW, scaling, init_sigma, a, b, start_lr):
    L.check(L.load().fd_vae_sample_add_noise(L.ptr(moments), L.ptr(post_eps), L.ptr(noise), L.ptr(out), HW, scaling,
                                             init_sigma, a, b, int(start_lr),
                                             L.dtype_code(moments.dtype) if moments is not None else 0, L.stream()),
            "fd_vae_sample_add_noise")
    return out


def postprocess_u8(x, out):
    L.check(L.load().fd_postprocess_u8(L.ptr(x), L.ptr(out), x.numel(), L.dtype_code(x.dtype), L.stream()),
            "fd_postprocess_u8")
    return out


def blend_edge(a, b, Ha, Wa, Hb, Wb, C, extent, vertical):
    L.check(L.load().fd_blend_edge(L.ptr(a), L.ptr(b), Ha, Wa, Hb, Wb, C, extent, int(vertical),
                                   L.dtype_code(b.dtype), L.stream()), "fd_blend_edge")
    return b


def copy_2d(src, src_ld, dst, dst_ld, rows, cols):
    """dst[r][0:cols] = src[r][0:cols] (element row strides src_ld / dst_ld)."""
    L.check(L.load().fd_add_strided(L.ptr(src), src_ld, None, 0, L.ptr(dst), dst_ld, rows, cols,
                                    L.dtype_code(src.dtype), L.dtype_code(dst.dtype), L.stream()), "fd_add_strided")
    return dst
