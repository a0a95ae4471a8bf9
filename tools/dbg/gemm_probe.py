"""Probe: fp32 rotation y = x A^T at 1M x 1536 — mivq_opq_rotate vs torch.mm (rocBLAS/hipBLASLt)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
from haag_vq import _native  # noqa: E402

dev = _native.require_device()
n, d = 1_000_000, 1536
x = torch.randn(n, d, device=dev)
A = torch.linalg.qr(torch.randn(d, d, device=dev))[0].contiguous()
torch.backends.cuda.matmul.allow_tf32 = False
for name, f in (("mivq_opq_rotate", lambda: _native.opq_rotate(x, A)), ("torch.mm fp32", lambda: torch.mm(x, A.t()))):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        y = f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 5
    print(f"{name:18s} {ms:8.3f} ms  {2 * n * d * d / ms / 1e9:8.1f} TFLOP/s", flush=True)
ya, yb = _native.opq_rotate(x, A), torch.mm(x, A.t())
yd = x.double() @ A.double().t()
print("max |err| vs fp64: mivq", float((ya.double() - yd).abs().max()), " torch", float((yb.double() - yd).abs().max()))
