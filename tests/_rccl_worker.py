"""Rank body of tests/test_sharded_gpu.py::test_rccl_collectives_world1 (not a test module).

Joins an RCCL ("nccl") process group of world size 1 on cuda:0 and runs, on device tensors,
every collective the multi-GPU path issues: the codebook / query broadcast
(`broadcast_`), the quantizer broadcast (`broadcast_object_list` with a device),
`all_gather_into_tensor` of per-rank sorted top-k lists followed by `mivq_topk_merge` (what
`exchange_topk` does at world > 1), the shard-size gather, and bench.py's max-over-ranks
`all_reduce`.  Writes the checks to argv[1] as JSON.  At world 1 every collective is the
identity, so each result must equal its input; the point is that RCCL initialises and runs
these calls on the box's GPU (the driver's 8-GPU run is the only multi-rank RCCL run)."""
import json
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))

from haag_vq import _native  # noqa: E402


def main():
    out = Path(sys.argv[1])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    g = torch.Generator(device=dev).manual_seed(5)

    C = torch.randn(16, 256, 96, device=dev, generator=g)
    C0 = C.clone()
    dist.broadcast(C, src=0)
    res["broadcast_equal"] = bool(torch.equal(C, C0))

    obj = [{"M": 16, "B": 8, "codebooks": C0[:1, :2, :3].cpu().tolist()}]
    dist.broadcast_object_list(obj, src=0, device=dev)
    res["object_equal"] = obj[0]["codebooks"] == C0[:1, :2, :3].cpu().tolist()

    nq, k = 64, 10
    d = torch.sort(torch.rand(nq, k, device=dev, generator=g), dim=1).values
    i = torch.randint(0, 1 << 20, (nq, k), device=dev, dtype=torch.int32, generator=g)
    gd = torch.empty((nq, k), dtype=d.dtype, device=dev)
    gi = torch.empty((nq, k), dtype=i.dtype, device=dev)
    dist.all_gather_into_tensor(gd, d)
    dist.all_gather_into_tensor(gi, i)
    md, mi = _native.topk_merge(gd.view(1, nq, k), gi.view(1, nq, k), k)
    res["allgather_merge_equal"] = bool(torch.equal(md, d) and torch.equal(mi, i))

    sizes = torch.empty((1,), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes, torch.tensor([123457], dtype=torch.int64, device=dev))
    res["sizes"] = sizes.cpu().tolist()

    t = torch.tensor([1.25], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    res["allreduce_max"] = float(t.item())
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    out.write_text(json.dumps(res))


if __name__ == "__main__":
    main()
