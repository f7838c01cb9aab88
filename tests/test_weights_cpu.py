"""local weight ingestion through the drop-in factory, no GPU.

A diffusers-layout SDXL directory (unet/diffusion_pytorch_model.fp16.safetensors, text_encoder{,_2}/
model.fp16.safetensors), a VAE directory and a ``FaithDiff.bin`` holding the FaithDiff extras, the
``denoise_encoder.`` weights and an override of one core UNet weight (stage-2 checkpoints carry fine-tuned core
weights too) are written with seeded values; ``FaithDiff_pipeline(sdxl, vae, faithdiff)`` must load every
tensor bitwise, apply the reference's prefix split (unet_2d_condition_vae_extension.py:444-478: core
non-strict, each extras group strict; create_FaithDiff_model.py:13-22) and raise on strict-extras mismatches.
``FaithDiff.bin`` is read with torch.load(weights_only=True) (the reference's weights_only=False pickle load at
ext:427 is deliberately not reproduced)."""
import os

import pytest
import torch
from safetensors.torch import save_file

from fdhip import arch

EXTRA = ("information_transformer_layes.", "condition_embedding.", "spatial_ch_projs.")


def _fp16(shapes, seed):
    return {k: v.contiguous() for k, v in arch.random_init(shapes, seed=seed, dtype=torch.float16).items()}


@pytest.fixture(scope="module")
def weights(tmp_path_factory):
    root = tmp_path_factory.mktemp("weights")
    sdxl, vae_dir, fd_dir = root / "sdxl", root / "vae", root / "fd"
    for d in (sdxl / "unet", sdxl / "text_encoder", sdxl / "text_encoder_2", vae_dir, fd_dir):
        d.mkdir(parents=True)
    unet = _fp16(arch.unet_param_shapes(with_extras=False), 101)
    save_file(unet, str(sdxl / "unet" / "diffusion_pytorch_model.fp16.safetensors"))
    te = _fp16(arch.clip_param_shapes(arch.CLIP_L), 102)
    save_file(te, str(sdxl / "text_encoder" / "model.fp16.safetensors"))
    te2 = _fp16(arch.clip_param_shapes(arch.CLIP_G), 103)
    save_file(te2, str(sdxl / "text_encoder_2" / "model.fp16.safetensors"))
    vae = _fp16(arch.vae_param_shapes(), 104)
    save_file(vae, str(vae_dir / "diffusion_pytorch_model.safetensors"))
    ext = {k: v for k, v in arch.unet_param_shapes(True).items() if k.startswith(EXTRA)}
    fd = _fp16({**ext, **arch.encoder_param_shapes("denoise_encoder.", with_out=False)}, 105)
    fd["conv_in.weight"] = (unet["conv_in.weight"].float() * -2.0).half()  # a fine-tuned core weight
    torch.save(fd, str(fd_dir / "FaithDiff.bin"))
    del te, te2
    return dict(sdxl=str(sdxl), vae=str(vae_dir), fd=str(fd_dir), unet=unet, vae_sd=vae, fd_sd=fd)


def _same(a, b):
    return a.dtype == b.dtype and a.shape == b.shape and torch.equal(a, b)


def test_factory_loads_local_diffusers_layout_bitwise(weights):
    from FaithDiff.create_FaithDiff_model import FaithDiff_pipeline
    pipe = FaithDiff_pipeline(weights["sdxl"], weights["vae"], weights["fd"])
    usd = pipe.unet._sd
    fd = weights["fd_sd"]
    for k, v in weights["unet"].items():
        want = fd[k] if k in fd else v  # FaithDiff.bin's core keys override the SDXL unet (non-strict core load)
        assert _same(usd[k], want), k
    for k, v in fd.items():
        if k.startswith(EXTRA):
            assert _same(usd[k], v), k
    den = pipe.unet.denoise_encoder._sd
    n_den = 0
    for k, v in fd.items():
        if k.startswith("denoise_encoder."):
            assert _same(den[k[len("denoise_encoder."):]], v), k
            n_den += 1
    assert n_den == len(arch.encoder_param_shapes("", with_out=False)) and len(den) == n_den
    for k, v in weights["vae_sd"].items():
        assert _same(pipe.vae._sd[k], v), k
    assert pipe.text_encoder._sd.keys() == set(arch.clip_param_shapes(arch.CLIP_L))
    assert arch.count(arch.clip_param_shapes(arch.CLIP_G)) == sum(t.numel() for t in pipe.text_encoder_2._sd.values())
    assert pipe.unet.information_transformer_layes and pipe.unet.condition_embedding and pipe.unet.spatial_ch_projs


def _fd_variant(weights, tmp_path, edit):
    fd = dict(weights["fd_sd"])
    edit(fd)
    p = tmp_path / "FaithDiff.bin"
    torch.save(fd, str(p))
    return str(p)


@pytest.mark.parametrize("case", ["missing_extra", "unexpected_extra", "bad_shape_core", "bad_shape_encoder"])
def test_strict_extras_and_shape_mismatch_raise(weights, tmp_path, case):
    from FaithDiff.models.unet_2d_condition_vae_extension import UNet2DConditionModel
    edits = {
        "missing_extra": lambda fd: fd.pop("information_transformer_layes.1.mlp.c_fc.weight"),
        "unexpected_extra": lambda fd: fd.__setitem__("condition_embedding.extra.weight", torch.zeros(3)),
        "bad_shape_core": lambda fd: fd.__setitem__("conv_in.weight", torch.zeros(320, 4, 1, 1, dtype=torch.float16)),
        "bad_shape_encoder": lambda fd: fd.__setitem__("denoise_encoder.conv_in.weight",
                                                       torch.zeros(128, 3, 1, 1, dtype=torch.float16)),
    }
    path = _fd_variant(weights, tmp_path, edits[case])
    unet = UNet2DConditionModel(weights["unet"])
    with pytest.raises(RuntimeError):
        unet.load_additional_layers(weight_path=path)


def test_core_keys_are_non_strict(weights, tmp_path):
    """A FaithDiff.bin without core keys (stage-1 checkpoints hold only the extras) loads; so does one with a
    subset of them."""
    from FaithDiff.models.unet_2d_condition_vae_extension import UNet2DConditionModel
    path = _fd_variant(weights, tmp_path, lambda fd: fd.pop("conv_in.weight"))
    unet = UNet2DConditionModel(dict(weights["unet"]))
    unet.load_additional_layers(weight_path=path)
    assert _same(unet._sd["conv_in.weight"], weights["unet"]["conv_in.weight"])


def test_missing_local_weights_raise(tmp_path):
    from FaithDiff.models.unet_2d_condition_vae_extension import UNet2DConditionModel
    with pytest.raises(FileNotFoundError):
        UNet2DConditionModel.from_pretrained(str(tmp_path), subfolder="unet", variant="fp16")


def test_pickle_payloads_are_refused(weights, tmp_path):
    """weights_only=True: a FaithDiff.bin that needs arbitrary unpickling is rejected, not executed."""
    import pickle

    class Payload:
        def __reduce__(self):
            return (os.getcwd, ())

    p = tmp_path / "FaithDiff.bin"
    with open(p, "wb") as f:
        pickle.dump({"x": Payload()}, f)
    from FaithDiff.models.unet_2d_condition_vae_extension import UNet2DConditionModel
    unet = UNet2DConditionModel(dict(weights["unet"]))
    with pytest.raises(Exception):
        unet.load_additional_layers(weight_path=str(p))


def _pipe_digest(pipe):
    """{component: {key: (dtype, shape, crc32 of the bytes)}} over every weight the pipeline holds."""
    import zlib
    out = {}
    for name, m in pipe._weight_owners():
        if m is None:
            continue
        out[name] = {k: (str(v.dtype), tuple(v.shape), zlib.crc32(v.detach().contiguous().view(torch.uint8).numpy()))
                     for k, v in m._sd.items()}
    return out


def _collective_build_worker(rank, world, port, paths, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from FaithDiff.create_FaithDiff_model import FaithDiff_pipeline
        # only rank 0 may read: every other rank gets paths that do not exist, so any read would raise
        p = paths if rank == 0 else ("/nonexistent/sdxl", "/nonexistent/vae", "/nonexistent/fd")
        pipe = FaithDiff_pipeline(*p, process_group=dist.group.WORLD)
        q.put((rank, _pipe_digest(pipe), pipe.last_broadcast_bytes))
    finally:
        dist.destroy_process_group()


def test_collective_build_only_rank0_reads(weights):
    """FaithDiff_pipeline(..., process_group=WORLD) on 2 gloo ranks: rank 0 reads the local diffusers checkpoints, rank
    1 reads nothing (its paths do not exist) and receives every weight by broadcast (manifest + dtype buckets,
    tile_parallel.broadcast_state_dict) -- both end with the same keys, dtypes, shapes and bytes, which are the files'
    (create_FaithDiff_model.py:13-22 loads them in every process instead)."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    paths = (weights["sdxl"], weights["vae"], weights["fd"])
    procs = [ctx.Process(target=_collective_build_worker, args=(r, 2, port, paths, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (_, d0, n0), (_, d1, n1) = res
    assert d0 == d1 and n0 == n1 > 5e9
    import zlib
    want = weights["vae_sd"]["decoder.conv_in.weight"]
    assert d0["vae"]["decoder.conv_in.weight"][2] == zlib.crc32(want.contiguous().view(torch.uint8).numpy())
