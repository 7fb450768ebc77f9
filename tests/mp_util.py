"""Passing tensors from spawned test workers to the parent by value.

A CPU tensor put on a multiprocessing queue travels as a shared-memory file descriptor that the
parent fetches from the child's resource-sharer socket when it unpickles the item; a worker that
has already exited by then leaves the parent with ``FileNotFoundError``.  Workers send
``to_np(obj)`` (numpy arrays pickle by value) and the parent restores tensors with ``to_torch``.
"""
from __future__ import annotations

import numpy as np
import torch


def to_np(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().numpy()
    if isinstance(obj, (list, tuple)):
        return type(obj)(to_np(o) for o in obj)
    if isinstance(obj, dict):
        return {k: to_np(v) for k, v in obj.items()}
    return obj


def to_torch(obj):
    if isinstance(obj, np.ndarray):
        return torch.from_numpy(obj)
    if isinstance(obj, (list, tuple)):
        return type(obj)(to_torch(o) for o in obj)
    if isinstance(obj, dict):
        return {k: to_torch(v) for k, v in obj.items()}
    return obj
