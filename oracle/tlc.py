"""Restatement of the TLC latent-tile loop helper ``LocalAttention``.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
Follows FaithDiff/pipelines/pipeline_FaithDiff_tlc.py:
  * grids ............ :160-205 (k clamped to h,w; step ceil(k*overlap) unless a single row/col;
                       last tile snapped to the edge)
  * _gaussian_weights  :207-228 (fp64; x midpoint (W-1)/2 but y midpoint H/2; tiled to 4 channels)
  * grids_inverse .... :230-252 (fp32 canvas, tile order, unclamped kernel_size slicing)
Pinned against vectors generated from the reference (tests/golden/make_golden.py).
"""
import math

import numpy as np
import torch


def tile_origins(h, w, kernel_size, overlap):
    k1, k2 = kernel_size
    k1 = min(k1, h)
    k2 = min(k2, w)
    num_row = (h - 1) // k1 + 1
    num_col = (w - 1) // k2 + 1
    step_j = k2 if num_col == 1 else math.ceil(k2 * overlap)
    step_i = k1 if num_row == 1 else math.ceil(k1 * overlap)
    idx = []
    i, last_i = 0, False
    while i < h and not last_i:
        j = 0
        if i + k1 >= h:
            i = h - k1
            last_i = True
        last_j = False
        while j < w and not last_j:
            if j + k2 >= w:
                j = w - k2
                last_j = True
            idx.append((i, j))
            j = j + step_j
        i = i + step_i
    return idx, (k1, k2)


def gaussian_weights(tile_width, tile_height):
    var = 0.01
    mid = (tile_width - 1) / 2
    xp = [np.exp(-(x - mid) * (x - mid) / (tile_width * tile_width) / (2 * var)) / np.sqrt(2 * np.pi * var)
          for x in range(tile_width)]
    mid = tile_height / 2
    yp = [np.exp(-(y - mid) * (y - mid) / (tile_height * tile_height) / (2 * var)) / np.sqrt(2 * np.pi * var)
          for y in range(tile_height)]
    return torch.tile(torch.tensor(np.outer(yp, xp)), (4, 1, 1))


class LocalAttention:
    def __init__(self, kernel_size, overlap=0.5):
        self.kernel_size = kernel_size
        self.overlap = overlap

    def grids(self, x):
        b, c, h, w = x.shape
        assert b == 1
        self.original_size = (b, c, h, w)
        idx, (k1, k2) = tile_origins(h, w, self.kernel_size, self.overlap)
        self.tile_weights = gaussian_weights(k2, k1)
        self.idxes = [{"i": i, "j": j} for i, j in idx]
        return torch.cat([x[:, :, i:i + k1, j:j + k2] for i, j in idx], dim=0)

    def grids_inverse(self, outs):
        b, c, h, w = self.original_size
        preds = torch.zeros(self.original_size)
        count = torch.zeros((b, 4, h, w))
        k1, k2 = self.kernel_size
        for cnt, e in enumerate(self.idxes):
            i, j = e["i"], e["j"]
            preds[0, :, i:i + k1, j:j + k2] += outs[cnt] * self.tile_weights
            count[0, :, i:i + k1, j:j + k2] += self.tile_weights
        return preds / count
