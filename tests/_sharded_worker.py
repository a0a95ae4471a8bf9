"""Rank body of tests/test_sharded_gpu.py::test_sharded_flat_index_two_ranks_one_gpu (run under
torch.distributed.run; not a test module).  Every rank holds one row shard of the same seeded
database in a ShardedFlatIndex; rank 0 also ranks the whole database with the broadcast
quantizer on one device and writes both answers to argv[1] as JSON."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))

from haag_vq.methods.product_quantization import ProductQuantizer  # noqa: E402
from haag_vq.methods.search.flat_quantized_index import search_codes  # noqa: E402
from haag_vq.parallel.launch import finish_rank, init_rank  # noqa: E402
from haag_vq.parallel.sharded import ShardedFlatIndex, shard_range  # noqa: E402


def main():
    out = Path(sys.argv[1])
    info = init_rank()
    n, d, nq, k = 30011, 64, 40, 10
    X = np.random.default_rng(3).standard_normal((n, d)).astype(np.float32)
    X[17] = X[5]  # an exact duplicate: distance ties across the shard boundary are ordered by id
    X[n - 3] = X[5]
    Q = np.random.default_rng(4).standard_normal((nq, d)).astype(np.float32)
    Q[0] = X[5]
    a, b = shard_range(n, info.rank, info.world)
    res = {}
    for metric in ("l2", "ip"):
        idx = ShardedFlatIndex(ProductQuantizer(M=8, B=8))
        idx.fit(X[a:b], metric=metric, train=X[:8192] if info.rank == 0 else None)
        ids, dists = idx.search_with_scores(Q, k)
        if info.rank == 0:
            codes = idx.quantizer.compress(torch.from_numpy(X).cuda())
            d1, i1 = search_codes(idx.quantizer, codes, Q, k, metric)
            res[metric] = {"sharded_ids": ids.astype(np.int64).tolist(), "sharded_d": dists.tolist(),
                           "single_ids": i1.cpu().numpy().view(np.uint32).astype(np.int64).tolist(),
                           "single_d": d1.cpu().numpy().tolist()}
        idx.save(out.parent / f"idx_{metric}")  # per-rank shard files, then a fresh index from them
        idx2 = ShardedFlatIndex(ProductQuantizer(M=8, B=8))
        idx2.load(out.parent / f"idx_{metric}")
        ids2, dists2 = idx2.search_with_scores(Q, k)
        if info.rank == 0:
            res[metric]["reload_equal"] = bool(np.array_equal(ids2, ids) and np.array_equal(dists2, dists))
        big = idx.search_with_scores(Q[:3], 300)  # k > 256: the decode + exact path per shard
        if info.rank == 0:
            res[metric]["k300_ids"] = big[0].astype(np.int64).tolist()
            d3, i3 = search_codes(idx.quantizer, codes, Q[:3], 300, metric)
            res[metric]["k300_single_ids"] = i3.cpu().numpy().view(np.uint32).astype(np.int64).tolist()
    if info.rank == 0:
        res["world"] = info.world
        out.write_text(json.dumps(res))
    finish_rank(info)


if __name__ == "__main__":
    main()
