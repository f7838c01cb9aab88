"""Drop-in for FaithDiff/models/bsrnet_arch.py (RRDBNet, :77-175): the BSRNet degradation-removal pre-pass that
test.py:97-101 runs before the LLaVA caption, on the HIP path (fdhip/bsrnet.py).

Same constructor, state-dict keys (strict load), forward(x) on NCHW [1, 3, H, W] images in [0, 1] -> [1, 3, 4H, 4W]
and deg_remove(input, tile_size=512, tile_pad=16).  Only the published configuration is supported (in_nc = out_nc
= 3, nf = 64, gc = 32, sf = 4; nb free).  There is no CPU path: forward needs .to('cuda') and a gfx950 device.
"""
import torch

from fdhip import arch


class RRDBNet:
    def __init__(self, in_nc=3, out_nc=3, nf=64, nb=23, gc=32, sf=4):
        if (in_nc, out_nc, nf, gc, sf) != (3, 3, 64, 32, 4):
            raise NotImplementedError("BSRNet on HIP: only in_nc=out_nc=3, nf=64, gc=32, sf=4 (the published model)")
        self.nb, self.sf, self.scale_factor = nb, sf, 4
        self._shapes = arch.bsrnet_param_shapes(nb)
        self._sd = None
        self._hip = None
        self._device = torch.device("cpu")

    def load_state_dict(self, sd, strict=True):
        missing = [k for k in self._shapes if k not in sd]
        unexpected = [k for k in sd if k not in self._shapes]
        bad = [k for k in self._shapes if k in sd and tuple(sd[k].shape) != self._shapes[k]]
        if bad or (strict and (missing or unexpected)):
            raise RuntimeError(f"Error(s) in loading state_dict for RRDBNet: missing={missing[:5]} "
                               f"unexpected={unexpected[:5]} shape mismatch={bad[:5]}")
        if missing:
            raise RuntimeError(f"RRDBNet: no weights for {missing[:5]}")
        self._sd = {k: sd[k].detach().to("cpu", torch.float32) for k in self._shapes}
        self._hip = None
        return [], unexpected

    def state_dict(self):
        return dict(self._sd or {})

    def to(self, device=None, dtype=None, **kwargs):
        if isinstance(device, torch.dtype):
            device = None
        if device is not None:
            self._device = torch.device(device)
            if self._device.type == "cuda" and self._device.index is None:
                self._device = torch.device("cuda", torch.cuda.current_device())
            self._hip = None
        return self

    def eval(self):
        return self

    def hip(self):
        if self._hip is None:
            if self._sd is None:
                raise RuntimeError("RRDBNet: load_state_dict first")
            if self._device.type != "cuda":
                raise RuntimeError("BSRNet runs only on an MI355X (gfx950); call .to('cuda') first")
            from fdhip.bsrnet import HipRRDBNet
            self._hip = HipRRDBNet(self._sd, self.nb, self._device)
        return self._hip

    def __call__(self, x):
        return self.forward(x)

    def forward(self, x):
        return self.hip().forward(x)

    @torch.no_grad()
    def deg_remove(self, input, tile_size=512, tile_pad=16):
        return self.hip().deg_remove(input, tile_size, tile_pad)


BSRNet = RRDBNet
