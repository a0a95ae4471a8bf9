"""`vq-benchmark precompute-gt`: exact k-nearest neighbours (L2) of the first ``num_queries``
vectors of a ``.npy`` file against all of them, saved as ``<output>.npy`` (int64 ids) and
``<output>.distances.npy`` (float32 squared distances) for ``sweep --ground-truth-path``.

Mirrors /root/reference/src/haag_vq/benchmarks/precompute_ground_truth.py:14-129 (SURVEY §8f
rank 3).  The reference builds a faiss IndexFlatL2 on the whole array; here the file is
memory-mapped (``allow_pickle=False``) and the database is streamed to the device in row
slices, each searched with ``mivq_flat_search`` and the per-slice lists merged with
``mivq_topk_merge`` (deterministic (distance, id) order), so the host holds one slice beyond
the mapping and the device one slice plus the queries.  ``--use-gpu`` is accepted for the reference's
command line; the search always runs on the MI355X.
"""

from __future__ import annotations

from pathlib import Path
from time import perf_counter

import numpy as np
import typer

# rows of the database per device slice (about 1.5 GB of fp32 at D = 1536)
_SLICE_ROWS = 1 << 18


def exact_knn_l2(vectors: np.ndarray, queries: np.ndarray, k: int, batch_size: int = 1000,
                 slice_rows: int = _SLICE_ROWS):
    """(ids int64 (nq, k), squared L2 distances float32 (nq, k)), best first.

    k > len(vectors) keeps the requested width, as faiss IndexFlatL2.search does: the columns
    past the database hold id -1 and distance FLT_MAX (faiss's CMax heap neutral; faiss is not
    importable here, so the pad value is parity-unpinned)."""
    import torch

    from haag_vq import _arrays, _native

    n = vectors.shape[0]
    nq = queries.shape[0]
    k_req = int(k)
    ids_out = np.full((nq, k_req), -1, dtype=np.int64)
    dist_out = np.full((nq, k_req), np.finfo(np.float32).max, dtype=np.float32)
    k = min(k_req, n)
    if nq == 0 or k == 0:
        return ids_out, dist_out
    Qd = _arrays.to_device(np.array(queries, dtype=np.float32, copy=True))
    parts_d, parts_i = [], []
    for s in range(0, n, slice_rows):
        # a writable host copy of the slice (torch refuses to wrap a read-only memory map)
        Xs = _arrays.to_device(np.array(vectors[s:s + slice_rows], dtype=np.float32, copy=True))
        kk = min(k, Xs.shape[0])
        d_b, i_b = [], []
        for q0 in range(0, nq, batch_size):
            d, i = _native.flat_search(Qd[q0:q0 + batch_size], Xs, kk, id_offset=s)
            d_b.append(d)
            i_b.append(i)
        d, i = torch.cat(d_b), torch.cat(i_b)
        if kk < k:  # a short last slice: pad with +inf so the merge never picks the pads
            d = torch.cat([d, torch.full((nq, k - kk), float("inf"), device=d.device)], 1)
            i = torch.cat([i, torch.full((nq, k - kk), -1, dtype=i.dtype, device=i.device)], 1)
        parts_d.append(d)
        parts_i.append(i)
        del Xs
    if len(parts_d) == 1:
        d, i = parts_d[0], parts_i[0]
    else:
        d, i = _native.topk_merge(torch.stack(parts_d).contiguous(), torch.stack(parts_i).contiguous(), k)
    ids_out[:, :k] = _arrays.to_host(i).view(np.uint32).astype(np.int64)
    dist_out[:, :k] = _arrays.to_host(d)
    return ids_out, dist_out


def precompute_ground_truth(
    vectors_path: str = typer.Option(..., help="Path to vectors file (.npy format)"),
    output_path: str = typer.Option(..., help="Path to save ground truth (.npy format)"),
    num_queries: int = typer.Option(100, help="Number of queries (taken from start of vectors)"),
    k: int = typer.Option(100, help="Number of nearest neighbors to compute"),
    use_gpu: bool = typer.Option(False, help="Accepted for compatibility; the search runs on the GPU"),
    batch_size: int = typer.Option(1000, help="Batch size for processing queries"),
):
    """Precompute exact k-nearest neighbours (L2) of the first num_queries vectors."""
    src = Path(vectors_path)
    if not src.exists():
        print(f"ERROR: Vectors file not found: {src}")
        raise typer.Exit(1)
    vectors = np.load(src, mmap_mode="r", allow_pickle=False)
    n, d = vectors.shape
    print(f"Loaded {n} vectors of dimension {d} from {src}")
    if num_queries > n:
        print(f"WARNING: num_queries ({num_queries}) > dataset size ({n})")
        num_queries = n
    t0 = perf_counter()
    ids, dists = exact_knn_l2(vectors, np.asarray(vectors[:num_queries]), k, batch_size=batch_size)
    dt = perf_counter() - t0
    print(f"Exact {k}-NN of {num_queries} queries in {dt:.2f}s "
          f"({dt / max(num_queries, 1) * 1e3:.2f} ms per query, mivq_flat_search)")
    out = Path(output_path)
    out.parent.mkdir(parents=True, exist_ok=True)
    np.save(out, ids)
    dpath = out.with_suffix(".distances.npy")
    np.save(dpath, dists)
    print(f"Saved ground truth {ids.shape} to {out} and distances to {dpath}")
    print(f"Use it with: vq-benchmark sweep --ground-truth-path {out}")
