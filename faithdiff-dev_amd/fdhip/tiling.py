"""Tiled VAE encode/decode and tiled denoise-encoder -- filled in below."""


def tiled_encoder_forward(enc, x, H, W):
    raise NotImplementedError("tiled denoise encoder: not built yet")


def tiled_vae_encode(vae, x, H, W):
    raise NotImplementedError("tiled VAE encode: not built yet")


def tiled_vae_decode(vae, z, h, w):
    raise NotImplementedError("tiled VAE decode: not built yet")
