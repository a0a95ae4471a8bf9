"""numpy / torch boundary helpers.

The reference API is numpy-in / numpy-out (inputs are copied to
C-contiguous f32, outputs are new caller-owned arrays).  The MI355X build keeps that
contract and additionally accepts device tensors, which stay resident (no host round
trip) — the form bench.py and the sharded path use.
"""

from __future__ import annotations

from typing import Iterator, Tuple

import numpy as np
import torch

from . import _native

# host -> device staging granularity for numpy inputs (bounded device footprint)
STAGE_BYTES = 1 << 31


def is_tensor(x) -> bool:
    return isinstance(x, torch.Tensor)


def device() -> torch.device:
    return _native.require_device()


def to_device(x, dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """Contiguous device tensor of `dtype` (copies numpy / host tensors)."""
    dev = device()
    if isinstance(x, torch.Tensor):
        t = x
        if t.device != dev or t.dtype != dtype:
            t = t.to(device=dev, dtype=dtype)
        return t.contiguous()
    a = np.ascontiguousarray(np.asarray(x), dtype=torch.empty((), dtype=dtype).numpy().dtype)
    return torch.from_numpy(a).to(dev)


def to_host(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


def row_chunks(n: int, row_bytes: int, max_bytes: int = STAGE_BYTES) -> Iterator[Tuple[int, int]]:
    step = max(1, int(max_bytes // max(1, row_bytes)))
    for s in range(0, n, step):
        yield s, min(n, s + step)
