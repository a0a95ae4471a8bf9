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
test_exchange_topk_gloo_world2_matches_single_rank, tests/test_bench_launcher.py), and over
gloo on host copies of device lists when several ranks share one GPU
(tests/test_sharded_gpu.py).

Callers: ``bench.py --gpus N`` (BASELINE config #5), ``vq-benchmark streaming-sweep --gpus N``
(benchmarks/streaming_sweep.py: row-sharded stream encode) and ``ShardedFlatIndex`` below
(the row-sharded ``FlatQuantizedIndex``).
"""

from __future__ import annotations

from pathlib import Path
from typing import Callable, Literal, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .. import _arrays, _native
from ..methods.base_quantizer import BaseQuantizer
from ..methods.base_search_index import BaseSearchIndex


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
    """In-place broadcast from ``src``; under gloo a device tensor goes through a host copy."""
    if _world()[1] > 1:
        if _host_collectives() and t.device.type != "cpu":
            h = t.cpu()
            dist.broadcast(h, src=src)
            t.copy_(h)
        else:
            dist.broadcast(t, src=src)
    return t


def _host_collectives() -> bool:
    return dist.get_backend() == "gloo"


def exchange_topk(d: torch.Tensor, i: torch.Tensor, k: int,
                  merge: Optional[Callable] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather per-rank sorted (nq, k) lists and merge them into the global top-k.

    Under RCCL the gather runs on the device lists; under gloo (CPU ranks, or several ranks
    sharing one GPU) on host copies, and the merge runs where the lists came from."""
    rank, world = _world()
    if world == 1:
        return d, i
    nq = d.shape[0]
    home = d.device
    if _host_collectives() and home.type != "cpu":
        d, i = d.cpu(), i.cpu()
    # output concatenated along dim 0 (the form every backend accepts), viewed per rank
    gd = torch.empty((world * nq, k), dtype=d.dtype, device=d.device)
    gi = torch.empty((world * nq, k), dtype=i.dtype, device=i.device)
    dist.all_gather_into_tensor(gd, d.contiguous())
    dist.all_gather_into_tensor(gi, i.contiguous())
    gd, gi = gd.to(home), gi.to(home)
    if merge is None and k > 256:
        merge = _merge_sorted_large  # mivq_topk_merge keeps its lists in one wave (k <= 256)
    merge = merge or _native.topk_merge
    return merge(gd.view(world, nq, k), gi.view(world, nq, k), k)


def _merge_sorted_large(gd: torch.Tensor, gi: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(parts, nq, k) lists -> (nq, k) by (dist, uint32 id), NaN as +inf: two stable sorts."""
    parts, nq, _ = gd.shape
    d = gd.permute(1, 0, 2).reshape(nq, parts * k)
    i = gi.permute(1, 0, 2).reshape(nq, parts * k)
    d = torch.where(torch.isnan(d), torch.full_like(d, float("inf")), d)
    iu = i.to(torch.int64) & 0xFFFFFFFF
    o1 = torch.argsort(iu, dim=1, stable=True)
    d1, i1 = torch.gather(d, 1, o1), torch.gather(i, 1, o1)
    o2 = torch.argsort(d1, dim=1, stable=True)[:, :k]
    return torch.gather(d1, 1, o2).contiguous(), torch.gather(i1, 1, o2).contiguous()


def broadcast_quantizer(model: Optional[BaseQuantizer], src: int = 0) -> BaseQuantizer:
    """Rank ``src``'s fitted quantizer on every rank (codebooks / rotation / SQ bounds as
    plain arrays, SURVEY §8e: trained once, broadcast once)."""
    from ..methods.search.flat_quantized_index import quantizer_from_state, quantizer_state

    rank, world = _world()
    if world == 1:
        return model
    obj = [quantizer_state(model) if rank == src else None]
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
    dist.broadcast_object_list(obj, src=src, device=dev)
    return model if rank == src else quantizer_from_state(obj[0])


def allgather_sizes(n_local: int) -> list:
    """Row counts of every rank's shard, in rank order."""
    rank, world = _world()
    if world == 1:
        return [int(n_local)]
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([int(n_local)], dtype=torch.int64, device=dev)
    g = torch.empty((world,), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(g, t)
    return [int(v) for v in g.cpu()]


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


class ShardedFlatIndex(BaseSearchIndex):
    """``FlatQuantizedIndex`` over a row-sharded database: one rank per GPU holds the codes of
    its own rows; search returns the global top-k (identical on every rank and for any number
    of ranks: ties go to the smaller global id).

    ``fit(X_local)``: rank 0 fits the quantizer on ``train`` (default: its own shard) and
    broadcasts it; every rank compresses its shard; global ids start at the sum of the lower
    ranks' shard sizes.  ``search_with_scores(Q, k)``: Q is taken from rank 0 (broadcast),
    every rank ranks its codes (``mivq_adc_search`` for PQ / OPQ, decode + exact for the rest)
    with its id offset, then one all-gather of the (nq, k) lists and the (dist, id) merge.
    Reference contract: /root/reference/src/haag_vq/methods/search/flat_quantized_index.py:34-76.
    """

    def __init__(self, quantizer: BaseQuantizer) -> None:
        self._quantizer = quantizer
        self._codes: Optional[torch.Tensor] = None
        self._metric: Literal["l2", "ip"] = "l2"
        self._N = 0
        self._n_local = 0
        self._offset = 0
        self._D = 0

    @property
    def quantizer(self) -> BaseQuantizer:
        return self._quantizer

    @property
    def id_offset(self) -> int:
        return self._offset

    def fit(self, X, metric: Literal["l2", "ip"] = "l2", train=None) -> None:
        from ..methods.search.flat_quantized_index import _METRIC

        if metric not in _METRIC:
            raise ValueError(f"metric must be 'l2' or 'ip', got {metric!r}")
        rank, _ = _world()
        Xd = _arrays.to_device(X, torch.float32)
        self._metric = metric
        self._n_local, self._D = Xd.shape
        if rank == 0:
            self._quantizer.fit(Xd if train is None else _arrays.to_device(train, torch.float32))
        self._quantizer = broadcast_quantizer(self._quantizer if rank == 0 else None)
        sizes = allgather_sizes(self._n_local)
        self._offset = int(sum(sizes[:rank]))
        self._N = int(sum(sizes))
        self._codes = self._quantizer.compress(Xd)

    def search(self, Q, k: int) -> np.ndarray:
        ids, _ = self.search_with_scores(Q, k)
        return ids

    def search_with_scores(self, Q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        from ..methods.search.flat_quantized_index import ids_to_numpy, search_codes

        Qd = broadcast_(_arrays.to_device(Q, torch.float32).contiguous())
        nq = Qd.shape[0]
        k = min(int(k), self._N)
        if k <= 0:
            return np.empty((nq, 0), dtype=np.uint32), np.empty((nq, 0), dtype=np.float32)
        kl = min(k, self._n_local)
        if kl > 0:
            d, i = search_codes(self._quantizer, self._codes, Qd, kl, self._metric, id_offset=self._offset)
        else:
            d = torch.empty((nq, 0), dtype=torch.float32, device=Qd.device)
            i = torch.empty((nq, 0), dtype=torch.int32, device=Qd.device)
        ip = self._metric == "ip"
        # pad a short shard with (+inf, 0xFFFFFFFF): never ahead of a real row in the merge
        if kl < k:
            d = torch.cat([d, torch.full((nq, k - kl), float("-inf") if ip else float("inf"), device=d.device)], 1)
            i = torch.cat([i, torch.full((nq, k - kl), -1, dtype=torch.int32, device=i.device)], 1)
        d = -d if ip else d  # the merge orders ascending
        d, i = exchange_topk(d.contiguous(), i.contiguous(), k)
        d = -d if ip else d
        return ids_to_numpy(i), _arrays.to_host(d)

    def memory_footprint(self) -> int:
        return int(self._codes.numel() * self._codes.element_size()) if self._codes is not None else 0

    # --------------------------------------------------------------- persistence
    @staticmethod
    def shard_path(path, rank: int, world: int) -> Path:
        """Each rank's file: <path>.rank<r>of<G>.npz (plain arrays, allow_pickle=False)."""
        return Path(f"{path}.rank{rank}of{world}.npz")

    def save(self, path) -> None:
        from ..methods.search.flat_quantized_index import quantizer_state

        rank, world = _world()
        f = self.shard_path(path, rank, world)
        f.parent.mkdir(parents=True, exist_ok=True)
        st = {"codes": _arrays.to_host(self._codes), "metric": np.array(self._metric), "N": np.array(self._N),
              "n_local": np.array(self._n_local), "offset": np.array(self._offset), "D": np.array(self._D)}
        st.update(quantizer_state(self._quantizer))
        with open(f, "wb") as fh:
            np.savez(fh, **st)

    def load(self, path) -> None:
        from ..methods.search.flat_quantized_index import quantizer_from_state

        rank, world = _world()
        with np.load(self.shard_path(path, rank, world), allow_pickle=False) as z:
            self._quantizer = quantizer_from_state(z)
            self._codes = torch.from_numpy(np.array(z["codes"])).to(_arrays.device())
            self._metric = str(z["metric"])
            self._N, self._n_local = int(z["N"]), int(z["n_local"])
            self._offset, self._D = int(z["offset"]), int(z["D"])

    def reconstruction_mse(self, X, sample_ids: Optional[np.ndarray] = None) -> Optional[float]:
        """Per-element MSE of this rank's rows (X: the local shard)."""
        if self._codes is None:
            return None
        X = np.asarray(X, dtype=np.float32)
        ids = np.arange(self._n_local) if sample_ids is None else np.asarray(sample_ids)
        xh = _arrays.to_host(self._quantizer.decompress(self._codes[torch.from_numpy(ids.astype(np.int64))
                                                                   .to(self._codes.device)].contiguous()))
        return float(np.mean((X[ids] - xh.astype(np.float32)) ** 2))
