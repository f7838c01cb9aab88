"""Host side of the TLC latent-tile loop: tile origins and gaussian blend weights.

Semantics of LocalAttention (FaithDiff/pipelines/pipeline_FaithDiff_tlc.py:101-252): kernel clamped to
the latent (h, w); step ceil(k * overlap) (k when a single row/column); the last tile snapped to the
edge; tiles in row-major order over a Cartesian grid of row and column origins.  Weights
(:207-228): fp64, x midpoint (W-1)/2 but y midpoint H/2 (asymmetric), var 0.01.  The per-element
split / blend run on the device (fd_tlc_* kernels); only these O(#tiles) index lists are host work.
"""
import math

import numpy as np


def axis_origins(n, k, overlap):
    """Origins along one axis (the inner loop of LocalAttention.grids)."""
    k = min(k, n)
    num = (n - 1) // k + 1
    step = k if num == 1 else math.ceil(k * overlap)
    out, pos, last = [], 0, False
    while pos < n and not last:
        if pos + k >= n:
            pos = n - k
            last = True
        out.append(pos)
        pos += step
    return out, k


# widest activation per latent position in a UNet forward (the information transformer's c_fc output at the tile's
# full resolution, 1280 channels; the up blocks' concats are 960)
WIDEST_CHANNELS = 1280


def max_tile_batch(kh, kw, cfg=2):
    """Most tiles one UNet forward may carry: the widest activation (cfg * tiles * kh * kw rows x WIDEST_CHANNELS)
    stays below 2^31 elements, the range of the kernels' 32-bit element offsets (51 for 128^2 tiles with CFG)."""
    return max(1, ((1 << 31) - 1) // (cfg * kh * kw * WIDEST_CHANNELS))


def tile_batches(count, tb, balance=False):
    """(first tile, tile count) of each UNet forward over a rank's `count` tiles, at most `tb` per forward: full
    batches and a remainder, or with `balance` ceil(count / tb) batches whose sizes differ by at most one (the
    larger ones first).  Every tile's result is independent of the batch it rides in (the tile-batch bitwise tests)."""
    if count <= 0:
        return []
    if not balance:
        return [(c0, min(tb, count - c0)) for c0 in range(0, count, tb)]
    nb = -(-count // tb)
    q, r = divmod(count, nb)
    out, c0 = [], 0
    for b in range(nb):
        n = q + (1 if b < r else 0)
        out.append((c0, n))
        c0 += n
    return out


class TileGrid:
    def __init__(self, h, w, kernel_size, overlap=0.5):
        self.h, self.w = h, w
        self.rows, self.kh = axis_origins(h, kernel_size[0], overlap)
        self.cols, self.kw = axis_origins(w, kernel_size[1], overlap)
        self.idxes = [{"i": i, "j": j} for i in self.rows for j in self.cols]

    @property
    def ntiles(self):
        return len(self.rows) * len(self.cols)

    def origin(self, t):
        return self.rows[t // len(self.cols)], self.cols[t % len(self.cols)]

    def weights(self):
        """(kh, kw) float64, identical for each of the 4 latent channels."""
        var = 0.01
        W, H = self.kw, self.kh
        mid = (W - 1) / 2
        xp = [np.exp(-(x - mid) * (x - mid) / (W * W) / (2 * var)) / np.sqrt(2 * np.pi * var) for x in range(W)]
        mid = H / 2
        yp = [np.exp(-(y - mid) * (y - mid) / (H * H) / (2 * var)) / np.sqrt(2 * np.pi * var) for y in range(H)]
        return np.outer(yp, xp)
