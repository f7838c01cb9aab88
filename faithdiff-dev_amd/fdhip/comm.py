"""The two collectives of the multi-GPU path, over torch.distributed.

On the GPUs the backend is 'nccl' = RCCL over xGMI and device buffers go straight to the collective.
Under 'gloo' with device tensors (several ranks sharing one GPU in tests) the buffers are staged through
host memory.
"""
import torch.distributed as dist


def _staged(group, t):
    """gloo on device tensors (a debugging / one-GPU multi-rank configuration): stage through host memory.
    RCCL ('nccl') takes the device buffers directly over xGMI."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_into(buf, local, group=None):
    """dist.all_gather_into_tensor(buf, local) -- one collective; host-staged under gloo."""
    if _staged(group, local):
        hb = buf.cpu()
        dist.all_gather_into_tensor(hb, local.cpu(), group=group)
        buf.copy_(hb)
    else:
        dist.all_gather_into_tensor(buf, local, group=group)
    return buf


def broadcast(t, src, group=None):
    """dist.broadcast(t, src) (src = global rank) -- host-staged under gloo."""
    if _staged(group, t):
        h = t.cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src=src, group=group)
    return t
