"""Row-sharded encode + ADC search across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI):

* encode is embarrassingly parallel: rank r owns rows [r*n, (r+1)*n) of the database and
  encodes them locally — no collective on the encode path;
* codebooks / OPQ matrix and the query block are replicated with one broadcast each;
* ADC search: every rank ranks its shard (global id = shard offset + local row), then ONE
  all-gather of the (nq, k) (dist, id) lists, followed by the on-device k-way merge
  (``mivq_topk_merge``).  The merge orders by (dist, id), so the result is identical for
  1, 2, 4 or 8 GPUs.

The exchange is written against the ``torch.distributed`` API only, so the same code runs
over gloo on CPU tensors in the multi-process tests (tests/test_host_cpu.py::
test_exchange_topk_gloo_world2_matches_single_rank, tests/test_bench_launcher.py).
"""

from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from .. import _native


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous row shard of rank r: [r*ceil(N/G), min(N, (r+1)*ceil(N/G)))."""
    per = -(-n_total // world)
    a = min(n_total, rank * per)
    return a, min(n_total, a + per)


def _world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if _world()[1] > 1:
        dist.broadcast(t, src=src)
    return t


def exchange_topk(d: torch.Tensor, i: torch.Tensor, k: int,
                  merge: Optional[Callable] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather per-rank sorted (nq, k) lists and merge them into the global top-k."""
    rank, world = _world()
    if world == 1:
        return d, i
    nq = d.shape[0]
    # output concatenated along dim 0 (the form every backend accepts), viewed per rank
    gd = torch.empty((world * nq, k), dtype=d.dtype, device=d.device)
    gi = torch.empty((world * nq, k), dtype=i.dtype, device=i.device)
    dist.all_gather_into_tensor(gd, d.contiguous())
    dist.all_gather_into_tensor(gi, i.contiguous())
    merge = merge or _native.topk_merge
    return merge(gd.view(world, nq, k), gi.view(world, nq, k), k)


def sharded_adc_search(Q: torch.Tensor, C: torch.Tensor, codes_u8: torch.Tensor, nbits: int, k: int,
                       id_offset: int, metric: int = _native.METRIC_L2) -> Tuple[torch.Tensor, torch.Tensor]:
    """Global top-k of Q over all ranks' code shards (Q and C replicated)."""
    lut = _native.adc_lut(Q, C, nbits, metric)
    d, i = _native.adc_search(lut, codes_u8, k, nbits, id_offset=id_offset)
    return exchange_topk(d, i, k)


def sharded_exact_search(Q: torch.Tensor, X: torch.Tensor, k: int, id_offset: int,
                         metric: int = _native.METRIC_L2) -> Tuple[torch.Tensor, torch.Tensor]:
    d, i = _native.flat_search(Q, X, k, metric, id_offset=id_offset)
    return exchange_topk(d, i, k)
