"""isaacgym.gymtorch mirror: zero-copy interop between gymapi.Tensor and torch.

wrap_tensor returns the sim-owned persistent torch tensor itself (same storage
on every acquire: test10_servo_vecenv.py:372-374 vs :400; equal data addresses
in examples/interop_torch.py:136-142). unwrap_tensor makes a non-owning
descriptor of a caller tensor, read synchronously (in stream order) by set_*.
"""
import torch

from .gymapi import Tensor


def wrap_tensor(gym_tensor, offsets=None, counts=None):
    if not isinstance(gym_tensor, Tensor):
        raise TypeError("wrap_tensor expects a gymapi.Tensor")
    t = gym_tensor._t
    if offsets is not None or counts is not None:
        off = tuple(offsets) if offsets is not None else (0,) * t.dim()
        cnt = tuple(counts) if counts is not None else tuple(s - o for s, o in zip(t.shape, off))
        for d, (o, c) in enumerate(zip(off, cnt)):
            t = t.narrow(d, o, c)
    return t


def unwrap_tensor(torch_tensor):
    if not isinstance(torch_tensor, torch.Tensor):
        raise TypeError("unwrap_tensor expects a torch.Tensor")
    return Tensor(torch_tensor)
