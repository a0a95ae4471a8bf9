"""Diagnostic for tests/test_concurrency_gpu.py: which output of the two-thread run differs from
the serial one, and whether the inputs change underneath (run on the GPU box)."""
import sys
import threading

sys.path.insert(0, "vector-quantization_amd")
import torch  # noqa: E402

from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402

dev = torch.device("cuda:0")


def work(seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.randn((60_000, 768), device=dev, generator=g)
    X = X / X.norm(dim=1, keepdim=True)
    C = train_pq(X[:8192], 8, 8, niter=4, seed=seed).contiguous()
    A, _ = torch.linalg.qr(torch.randn((768, 768), device=dev, generator=g, dtype=torch.float64))
    return X, C, A.float().contiguous()


def run(X, C, A):
    prep = _native.pq_prepare(C, 8)
    codes = _native.pq_encode(X, C, prep, 8)
    oprep = _native.opq_prepare(A, False)
    Y = _native.opq_rotate_prepared(X, oprep)
    lut = _native.adc_lut(X[:64], C, 8)
    d, i = _native.adc_search(lut, codes, 10, 8)
    return dict(codes=codes, Y=Y, lut=lut, dists=d, ids=i, prep=prep)


inputs = [work(s) for s in (1, 2)]
torch.cuda.synchronize()
sums = [[t.double().sum().item() for t in inp] for inp in inputs]
ref = [{k: v.cpu() for k, v in run(*inp).items()} for inp in inputs]
ref2 = [{k: v.cpu() for k, v in run(*inp).items()} for inp in inputs]
for i in range(2):
    for k in ref[i]:
        if not torch.equal(ref[i][k], ref2[i][k]):
            print(f"serial run not reproducible: input {i} key {k}", flush=True)

bad = 0
for trial in range(8):
    results = [None, None]

    def worker(i):
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            out = None
            for _ in range(4):
                out = run(*inputs[i])
            s.synchronize()
            results[i] = {k: v.cpu() for k, v in out.items()}

    th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i in range(2):
        for k in ref[i]:
            if not torch.equal(results[i][k], ref[i][k]):
                a, b = results[i][k], ref[i][k]
                if a.dtype.is_floating_point:
                    diff = (a - b).abs()
                    idx = (diff > 0).nonzero()[:5].tolist()
                    print(f"trial {trial} input {i} {k}: {int((diff > 0).sum())} differ, max {diff.max().item():.3g}, "
                          f"at {idx}", flush=True)
                else:
                    nd = int((a != b).sum())
                    print(f"trial {trial} input {i} {k}: {nd} differ at {(a != b).nonzero()[:5].tolist()}", flush=True)
                bad += 1
    now = [[t.double().sum().item() for t in inp] for inp in inputs]
    if now != sums:
        print(f"trial {trial}: inputs changed {sums} -> {now}", flush=True)
print("bad", bad, flush=True)
