"""ctypes binding of libmivq.so — the MI355X HIP implementation of the hot path.

Every public function here takes torch tensors that already live on the current HIP
device, validates shape / dtype / contiguity on the host, and calls the matching C entry
point of ``include/mivq.h`` on the current torch stream.  There is no CPU fallback: on a
machine without a HIP device (or without the built library) every compute call raises.

The error mapping mirrors the reference's exceptions:
  MIVQ_ERR_INVALID     -> ValueError (AssertionError for "D must be divisible by M",
                          product_quantization.py:61-62)
  MIVQ_ERR_UNSUPPORTED -> ValueError
  MIVQ_ERR_HIP / _WORKSPACE -> RuntimeError
"""

from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Optional, Tuple

import torch  # noqa: F401  (must be imported before libmivq: they share libamdhip64.so.7)

_PKG_ROOT = Path(__file__).resolve().parent.parent  # vector-quantization_amd/
LIB_PATH = Path(os.environ.get("MIVQ_LIB", _PKG_ROOT / "lib" / "libmivq.so"))

MIVQ_OK = 0
MIVQ_ERR_INVALID = -1
MIVQ_ERR_UNSUPPORTED = -2
MIVQ_ERR_HIP = -3
MIVQ_ERR_WORKSPACE = -4
MIVQ_PQ_AUTO = 0
MIVQ_PQ_FORCE_EXACT = 1
MIVQ_PQ_LEGACY_MFMA = 2
MIVQ_PQ_LEGACY_EXACT = 4
METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
NO_ID = 0xFFFFFFFF

_c = ctypes
_vp, _i32, _i64, _u32, _sz = _c.c_void_p, _c.c_int32, _c.c_int64, _c.c_uint32, _c.c_size_t

# name -> (restype, argtypes); exactly the declarations of include/mivq.h
SIGNATURES = {
    "mivq_last_error": (_c.c_char_p, []),
    "mivq_abi_version": (_c.c_int, []),
    "mivq_device_info": (_c.c_int, [_c.c_int, _c.c_char_p, _c.POINTER(_i32), _c.POINTER(_i64), _c.POINTER(_i64)]),
    "mivq_pq_prep_bytes": (_sz, [_i32, _i32, _i32]),
    "mivq_pq_prepare": (_c.c_int, [_vp, _i32, _i32, _i32, _vp, _vp]),
    "mivq_pq_encode_workspace_bytes": (_sz, [_i64, _i32, _i32, _i32]),
    "mivq_pq_encode": (_c.c_int, [_vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp, _u32, _vp]),
    "mivq_pq_decode": (_c.c_int, [_vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp]),
    "mivq_pq_unpack": (_c.c_int, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "mivq_kmeans_update": (_c.c_int, [_vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "mivq_opq_rotate": (_c.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp]),
    "mivq_opq_prep_bytes": (_sz, [_i32]),
    "mivq_opq_prepare": (_c.c_int, [_vp, _i32, _i32, _vp, _vp]),
    "mivq_opq_rotate_workspace_bytes": (_sz, [_i64, _i32]),
    "mivq_opq_rotate_prepared": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _sz, _vp, _vp]),
    "mivq_opq_gram_workspace_bytes": (_sz, [_i64, _i32]),
    "mivq_opq_gram": (_c.c_int, [_vp, _vp, _i64, _i32, _vp, _sz, _vp, _vp]),
    "mivq_sq_encode_f32": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]),
    "mivq_sq_encode_f64": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]),
    "mivq_sq_decode_f32": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]),
    "mivq_sq_decode_f64": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]),
    "mivq_rabitq_encode": (_c.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp]),
    "mivq_rabitq_decode": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "mivq_rabitq_search_workspace_bytes": (_sz, [_i64, _i64, _i32, _i32]),
    "mivq_rabitq_search": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _i64, _i32, _i32, _i32, _i64, _vp, _sz, _vp, _vp,
                                      _vp]),
    "mivq_extrabitq_normalize": (_c.c_int, [_vp, _i32, _i64, _i32, _vp, _vp, _vp, _vp]),
    "mivq_extrabitq_quantize": (_c.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp, _vp]),
    "mivq_extrabitq_dequantize": (_c.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp]),
    "mivq_extrabitq_finish": (_c.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp, _vp]),
    "mivq_extrabitq_rotate": (_c.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp]),
    "mivq_adc_lut": (_c.c_int, [_vp, _i64, _i32, _i32, _i32, _vp, _i32, _vp, _vp]),
    "mivq_adc_search_workspace_bytes": (_sz, [_i64, _i64, _i32, _i32, _i32]),
    "mivq_adc_search": (_c.c_int, [_vp, _i64, _vp, _i64, _i32, _i32, _i32, _i64, _vp, _sz, _vp, _vp, _c.c_uint32,
                                   _vp]),
    "mivq_flat_search_workspace_bytes": (_sz, [_i64, _i64, _i32, _i32]),
    "mivq_flat_search": (_c.c_int, [_vp, _i64, _vp, _i64, _i32, _i32, _i32, _i64, _vp, _sz, _vp, _vp, _vp]),
    "mivq_topk_merge": (_c.c_int, [_vp, _vp, _i32, _i64, _i32, _vp, _vp, _vp]),
    "mivq_pairwise_distances": (_c.c_int, [_vp, _i64, _vp, _i64, _i32, _i32, _vp, _vp]),
    "mivq_topk_rows": (_c.c_int, [_vp, _i64, _i64, _i32, _vp, _vp, _vp]),
    "mivq_bucket_sort_workspace_bytes": (_sz, [_i64, _i32]),
    "mivq_bucket_sort": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _sz, _vp]),
    "mivq_centroid_update": (_c.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "mivq_ivf_residuals": (_c.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "mivq_gather_rows": (_c.c_int, [_vp, _i64, _vp, _i64, _vp, _vp]),
    "mivq_ivfpq_terms": (_c.c_int, [_vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mivq_ivfpq_search_workspace_bytes": (_sz, [_i64, _i32, _i32]),
    "mivq_ivfpq_search": (_c.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _i32,
                                     _vp, _sz, _vp, _vp, _vp]),
}

ABI_VERSION = 2  # MIVQ_ABI_VERSION of include/mivq.h the table above binds
_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


def load_library() -> ctypes.CDLL:
    """Load libmivq.so and bind every exported symbol (works without a GPU)."""
    global _lib
    with _lock:
        if _lib is None:
            if not LIB_PATH.exists():
                raise RuntimeError(
                    f"libmivq.so not found at {LIB_PATH}; build it with "
                    "`make -C vector-quantization_amd/csrc` (or __graft_entry__.build())"
                )
            lib = ctypes.CDLL(str(LIB_PATH))
            lib.mivq_abi_version.restype = ctypes.c_int
            if lib.mivq_abi_version() != ABI_VERSION:
                raise RuntimeError(f"{LIB_PATH} has ABI {lib.mivq_abi_version()}, this package binds ABI "
                                   f"{ABI_VERSION}: rebuild it (make -C vector-quantization_amd/csrc)")
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def require_device() -> torch.device:
    """The HIP device compute runs on; raises when none is visible (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError(
            "haag_vq (MI355X build) needs a HIP device: no GPU is visible and this "
            "implementation has no CPU fallback"
        )
    load_library()
    return torch.device("cuda", torch.cuda.current_device())


def _raise(rc: int) -> None:
    msg = load_library().mivq_last_error().decode(errors="replace")
    if rc == MIVQ_ERR_INVALID:
        if "divisible" in msg:
            raise AssertionError(msg)
        raise ValueError(msg)
    if rc == MIVQ_ERR_UNSUPPORTED:
        raise ValueError(msg)
    raise RuntimeError(msg)


def _call(name: str, *args) -> None:
    rc = getattr(load_library(), name)(*args)
    if rc != MIVQ_OK:
        _raise(rc)


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _check(t: torch.Tensor, name: str, dtype: torch.dtype, ndim: Optional[int] = None) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name}: tensor must live on the HIP device")
    if t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype} != {dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim}-D, got shape {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")


# ----------------------------------------------------------------- workspace
def kernel_source_hash() -> str:
    """sha256 (first 16 hex digits) of the library's sources (csrc/*.hip, csrc/*.h,
    include/mivq.h, in name order): stamps PMC-derived numbers with the build they describe."""
    import hashlib

    h = hashlib.sha256()
    csrc = _PKG_ROOT / "csrc"
    files = sorted(list(csrc.glob("*.hip")) + list(csrc.glob("*.h"))) + [_PKG_ROOT.parent / "include" / "mivq.h"]
    for f in files:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    """Scratch buffer for one library call (the library never allocates).

    Allocated per call from torch's caching allocator on the current stream: the block goes
    back to that stream's pool when the caller drops it, and torch hands it out again only
    to later work on the same stream, which is ordered after the kernels that used it.  No
    module-level cache, so nothing outlives the call or follows a destroyed stream's handle."""
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


# ----------------------------------------------------------------- device info
def device_info(device: int = 0) -> dict:
    name = ctypes.create_string_buffer(64)
    cus, lds, hbm = _i32(), _i64(), _i64()
    _call("mivq_device_info", device, name, ctypes.byref(cus), ctypes.byref(lds), ctypes.byref(hbm))
    return {"arch": name.value.decode(), "cus": cus.value, "lds_per_cu": lds.value, "hbm_bytes": hbm.value}


# ----------------------------------------------------------------- PQ
def pq_code_size(M: int, nbits: int) -> int:
    return (M * nbits + 7) // 8


def pq_prepare(centroids: torch.Tensor, nbits: int) -> torch.Tensor:
    """centroids (M, ksub, dsub) f32 -> prep bytes for pq_encode."""
    _check(centroids, "centroids", torch.float32, 3)
    M, ksub, dsub = centroids.shape
    if ksub != (1 << nbits):
        raise ValueError(f"centroids have ksub={ksub}, expected 2**{nbits}")
    d = M * dsub
    nb = load_library().mivq_pq_prep_bytes(d, M, nbits)
    prep = torch.empty(nb, dtype=torch.uint8, device=centroids.device)
    _call("mivq_pq_prepare", _ptr(centroids), d, M, nbits, _ptr(prep), _stream())
    return prep


def pq_encode(x: torch.Tensor, centroids: torch.Tensor, prep: torch.Tensor, nbits: int,
              exact: bool = False, out: Optional[torch.Tensor] = None, flags_extra: int = 0) -> torch.Tensor:
    _check(x, "x", torch.float32, 2)
    _check(centroids, "centroids", torch.float32, 3)
    n, d = x.shape
    M, ksub, dsub = centroids.shape
    if d != M * dsub:
        raise ValueError(f"x has d={d}, codebook expects {M * dsub}")
    cs = pq_code_size(M, nbits)
    if out is None:
        out = torch.empty((n, cs), dtype=torch.uint8, device=x.device)
    else:
        _check(out, "out", torch.uint8, 2)
        if tuple(out.shape) != (n, cs):
            raise ValueError(f"out shape {tuple(out.shape)} != {(n, cs)}")
    nb = load_library().mivq_pq_encode_workspace_bytes(n, d, M, nbits)
    ws = workspace(nb, x.device)
    flags = (MIVQ_PQ_FORCE_EXACT if exact else MIVQ_PQ_AUTO) | flags_extra
    _call("mivq_pq_encode", _ptr(x), n, d, M, nbits, _ptr(centroids), _ptr(prep), _ptr(ws), ws.numel(),
          _ptr(out), flags, _stream())
    return out


def pq_decode(codes: torch.Tensor, centroids: torch.Tensor, nbits: int,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _check(codes, "codes", torch.uint8, 2)
    _check(centroids, "centroids", torch.float32, 3)
    M, ksub, dsub = centroids.shape
    n = codes.shape[0]
    if codes.shape[1] != pq_code_size(M, nbits):
        raise ValueError(f"codes have {codes.shape[1]} bytes per row, expected {pq_code_size(M, nbits)}")
    d = M * dsub
    if out is None:
        out = torch.empty((n, d), dtype=torch.float32, device=codes.device)
    _call("mivq_pq_decode", _ptr(codes), n, d, M, nbits, _ptr(centroids), _ptr(out), _stream())
    return out


def pq_unpack(codes: torch.Tensor, M: int, nbits: int) -> torch.Tensor:
    _check(codes, "codes", torch.uint8, 2)
    n = codes.shape[0]
    out = torch.empty((n, M), dtype=torch.uint8, device=codes.device)
    _call("mivq_pq_unpack", _ptr(codes), n, M, nbits, _ptr(out), _stream())
    return out


def kmeans_update(x: torch.Tensor, assign: torch.Tensor, centroids: torch.Tensor,
                  counts: torch.Tensor) -> None:
    _check(x, "x", torch.float32, 2)
    _check(assign, "assign", torch.uint8, 2)
    _check(centroids, "centroids", torch.float32, 3)
    _check(counts, "counts", torch.int32, 2)
    n, d = x.shape
    M, ksub, dsub = centroids.shape
    _call("mivq_kmeans_update", _ptr(x), n, d, M, ksub, _ptr(assign), _ptr(centroids), _ptr(counts), _stream())


# ----------------------------------------------------------------- OPQ
def opq_rotate(x: torch.Tensor, A: torch.Tensor, transpose: bool = False,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _check(x, "x", torch.float32, 2)
    _check(A, "A", torch.float32, 2)
    n, d = x.shape
    if tuple(A.shape) != (d, d):
        raise ValueError(f"A must be ({d}, {d}), got {tuple(A.shape)}")
    if out is None:
        out = torch.empty_like(x)
    _call("mivq_opq_rotate", _ptr(x), n, d, _ptr(A), 1 if transpose else 0, _ptr(out), _stream())
    return out


def opq_backend(d: Optional[int] = None) -> str:
    """What the OPQ classes rotate with (for reports)."""
    return "opq_row_scale_kernel + opq_split_gemm_kernel: split-f16 MFMA GEMM, fp32 accuracy"


def opq_prepare(A: torch.Tensor, transpose: bool = False) -> Optional[torch.Tensor]:
    """Scaled f16 hi / lo image of op(A) for opq_rotate_prepared (None when d % 8 != 0)."""
    _check(A, "A", torch.float32, 2)
    d = A.shape[0]
    if tuple(A.shape) != (d, d):
        raise ValueError(f"A must be square, got {tuple(A.shape)}")
    nb = load_library().mivq_opq_prep_bytes(d)
    if nb == 0:
        return None
    prep = torch.empty(nb, dtype=torch.uint8, device=A.device)
    _call("mivq_opq_prepare", _ptr(A), d, 1 if transpose else 0, _ptr(prep), _stream())
    return prep


def opq_rotate_prepared(x: torch.Tensor, prep: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x . op(A) for the op(A) that `prep` was built from (opq_prepare)."""
    _check(x, "x", torch.float32, 2)
    _check(prep, "prep", torch.uint8, 1)
    n, d = x.shape
    if prep.numel() != load_library().mivq_opq_prep_bytes(d):
        raise ValueError(f"prep has {prep.numel()} bytes, not the image of a ({d}, {d}) matrix")
    if out is None:
        out = torch.empty_like(x)
    else:
        _check(out, "out", torch.float32, 2)
        if tuple(out.shape) != (n, d):
            raise ValueError(f"out shape {tuple(out.shape)} != {(n, d)}")
    ws = workspace(load_library().mivq_opq_rotate_workspace_bytes(n, d), x.device)
    _call("mivq_opq_rotate_prepared", _ptr(x), n, d, _ptr(prep), _ptr(ws), ws.numel(), _ptr(out), _stream())
    return out


def opq_gram(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """G = x^T y in fp64 (d, d) on the library's fp64 MFMA kernel (OPQ Procrustes step)."""
    _check(x, "x", torch.float32, 2)
    _check(y, "y", torch.float32, 2)
    if x.shape != y.shape:
        raise ValueError(f"opq_gram: x {tuple(x.shape)} and y {tuple(y.shape)} differ")
    n, d = x.shape
    G = torch.empty((d, d), dtype=torch.float64, device=x.device)
    ws = workspace(load_library().mivq_opq_gram_workspace_bytes(n, d), x.device)
    _call("mivq_opq_gram", _ptr(x), _ptr(y), n, d, _ptr(ws), ws.numel(), _ptr(G), _stream())
    return G


# ----------------------------------------------------------------- SQ
def sq_encode(x: torch.Tensor, lo: torch.Tensor, den: torch.Tensor, nbits: int) -> torch.Tensor:
    if x.dtype not in (torch.float32, torch.float64):
        raise ValueError(f"sq_encode: unsupported dtype {x.dtype}")
    _check(x, "x", x.dtype, 2)
    _check(lo, "lo", x.dtype, 1)
    _check(den, "den", x.dtype, 1)
    n, d = x.shape
    if lo.numel() != d or den.numel() != d:
        raise ValueError(f"sq_encode: min/max have {lo.numel()}/{den.numel()} entries, data has d={d}")
    if nbits == 16:
        out = torch.empty((n, d), dtype=torch.int16, device=x.device)
    elif nbits == 8:
        out = torch.empty((n, d), dtype=torch.uint8, device=x.device)
    elif nbits == 4:
        out = torch.empty((n, (d + 1) // 2), dtype=torch.uint8, device=x.device)
    else:
        raise ValueError(f"num_bits must be 4, 8, or 16, got {nbits}")
    fn = "mivq_sq_encode_f64" if x.dtype == torch.float64 else "mivq_sq_encode_f32"
    _call(fn, _ptr(x), n, d, _ptr(lo), _ptr(den), nbits, _ptr(out), _stream())
    return out


def sq_decode(codes: torch.Tensor, d: int, lo: torch.Tensor, den: torch.Tensor, nbits: int) -> torch.Tensor:
    if not codes.is_contiguous() or not codes.is_cuda:
        raise ValueError("codes must be a contiguous device tensor")
    n = codes.shape[0]
    dt = lo.dtype
    _check(lo, "lo", dt, 1)
    _check(den, "den", dt, 1)
    if lo.numel() != d or den.numel() != d:
        raise ValueError(f"sq_decode: min/max have {lo.numel()}/{den.numel()} entries, expected d={d}")
    want = {4: ((d + 1) // 2, (torch.uint8,)), 8: (d, (torch.uint8,)), 16: (d, (torch.int16, torch.uint16))}
    if nbits not in want:
        raise ValueError(f"num_bits must be 4, 8, or 16, got {nbits}")
    width, dtypes = want[nbits]
    if codes.dim() != 2 or codes.shape[1] != width or codes.dtype not in dtypes:
        raise ValueError(f"sq_decode: {nbits}-bit codes of d={d} must be ({n}, {width}) {dtypes[0]}, "
                         f"got {tuple(codes.shape)} {codes.dtype}")
    out = torch.empty((n, d), dtype=dt, device=codes.device)
    fn = "mivq_sq_decode_f64" if dt == torch.float64 else "mivq_sq_decode_f32"
    _call(fn, _ptr(codes), n, d, _ptr(lo), _ptr(den), nbits, _ptr(out), _stream())
    return out


# ----------------------------------------------------------------- RaBitQ
def rabitq_code_size(d: int) -> int:
    return (d + 7) // 8 + 8


def rabitq_encode(x: torch.Tensor, centroid: Optional[torch.Tensor], metric: int) -> torch.Tensor:
    _check(x, "x", torch.float32, 2)
    if centroid is not None:
        _check(centroid, "centroid", torch.float32, 1)
    n, d = x.shape
    out = torch.empty((n, rabitq_code_size(d)), dtype=torch.uint8, device=x.device)
    _call("mivq_rabitq_encode", _ptr(x), n, d, _ptr(centroid), metric, _ptr(out), _stream())
    return out


def rabitq_decode(codes: torch.Tensor, d: int, centroid: Optional[torch.Tensor]) -> torch.Tensor:
    _check(codes, "codes", torch.uint8, 2)
    if codes.shape[1] != rabitq_code_size(d):
        raise ValueError(f"codes have {codes.shape[1]} bytes per row, expected {rabitq_code_size(d)}")
    n = codes.shape[0]
    out = torch.empty((n, d), dtype=torch.float32, device=codes.device)
    _call("mivq_rabitq_decode", _ptr(codes), n, d, _ptr(centroid), _ptr(out), _stream())
    return out


def rabitq_search(codes: torch.Tensor, d: int, centroid: Optional[torch.Tensor], q: torch.Tensor, qb: int,
                  metric: int, k: int, id_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """IndexRaBitQ estimator search: (keys f32 (nq, k), ids int32 (nq, k) holding uint32 ids);
    L2 keys are distance estimates, IP keys negated inner-product estimates (ascending)."""
    _check(codes, "codes", torch.uint8, 2)
    _check(q, "q", torch.float32, 2)
    if centroid is not None:
        _check(centroid, "centroid", torch.float32, 1)
    if codes.shape[1] != rabitq_code_size(d) or q.shape[1] != d:
        raise ValueError(f"codes rows {codes.shape[1]} B / queries d={q.shape[1]} do not match d={d}")
    n, nq = codes.shape[0], q.shape[0]
    dists = torch.empty((nq, k), dtype=torch.float32, device=q.device)
    ids = torch.empty((nq, k), dtype=torch.int32, device=q.device)
    ws = workspace(load_library().mivq_rabitq_search_workspace_bytes(nq, n, d, k), q.device)
    _call("mivq_rabitq_search", _ptr(codes), n, d, _ptr(centroid), _ptr(q), nq, qb, metric, k, id_offset, _ptr(ws),
          ws.numel(), _ptr(dists), _ptr(ids), _stream())
    return dists, ids


# ----------------------------------------------------------------- Extended RaBitQ
def extrabitq_code_size(d: int, nbits: int) -> int:
    return (d * nbits + 7) // 8 + 8


def extrabitq_rotate(o: torch.Tensor, P: torch.Tensor, transpose: bool) -> torch.Tensor:
    """o . P (or o . P^T) in fp64 on the library's MFMA GEMM (extended_rabitq.py:140,196)."""
    _check(o, "o", torch.float64, 2)
    _check(P, "P", torch.float64, 2)
    n, d = o.shape
    if tuple(P.shape) != (d, d):
        raise ValueError(f"P shape {tuple(P.shape)} != {(d, d)}")
    out = torch.empty((n, d), dtype=torch.float64, device=o.device)
    _call("mivq_extrabitq_rotate", _ptr(o), n, d, _ptr(P), 1 if transpose else 0, _ptr(out), _stream())
    return out


def extrabitq_encode(x: torch.Tensor, c: torch.Tensor, P: torch.Tensor, levels: torch.Tensor,
                     nbits: int) -> torch.Tensor:
    """Codes of ExtendedRaBitQuantizer.compress (the o . P rotation on mivq_extrabitq_rotate)."""
    if x.dtype not in (torch.float32, torch.float64):
        raise ValueError(f"extrabitq: unsupported dtype {x.dtype}")
    _check(x, "x", x.dtype, 2)
    for t, nm in ((c, "c"), (levels, "levels")):
        _check(t, nm, torch.float64, 1)
    _check(P, "P", torch.float64, 2)
    n, d = x.shape
    o = torch.empty((n, d), dtype=torch.float64, device=x.device)
    nrm = torch.empty((n,), dtype=torch.float64, device=x.device)
    _call("mivq_extrabitq_normalize", _ptr(x), 1 if x.dtype == torch.float64 else 0, n, d, _ptr(c), _ptr(o),
          _ptr(nrm), _stream())
    s_raw = extrabitq_rotate(o, P, False)
    codes = torch.empty((n, extrabitq_code_size(d, nbits)), dtype=torch.uint8, device=x.device)
    _call("mivq_extrabitq_quantize", _ptr(s_raw), n, d, _ptr(levels), nbits, _ptr(nrm), _ptr(codes), _stream())
    return codes


def extrabitq_decode(codes: torch.Tensor, c: torch.Tensor, P: torch.Tensor, levels: torch.Tensor,
                     nbits: int) -> torch.Tensor:
    _check(codes, "codes", torch.uint8, 2)
    n = codes.shape[0]
    d = P.shape[0]
    if codes.shape[1] != extrabitq_code_size(d, nbits):
        raise ValueError(f"codes have {codes.shape[1]} bytes per row, expected {extrabitq_code_size(d, nbits)}")
    o_hat = torch.empty((n, d), dtype=torch.float64, device=codes.device)
    _call("mivq_extrabitq_dequantize", _ptr(codes), n, d, _ptr(levels), nbits, _ptr(o_hat), _stream())
    y = extrabitq_rotate(o_hat, P, True)
    out = torch.empty((n, d), dtype=torch.float32, device=codes.device)
    _call("mivq_extrabitq_finish", _ptr(y), n, d, _ptr(codes), nbits, _ptr(c), _ptr(out), _stream())
    return out


# ----------------------------------------------------------------- ADC / flat search
def adc_lut(q: torch.Tensor, centroids: torch.Tensor, nbits: int, metric: int = METRIC_L2) -> torch.Tensor:
    _check(q, "q", torch.float32, 2)
    _check(centroids, "centroids", torch.float32, 3)
    nq, d = q.shape
    M, ksub, dsub = centroids.shape
    if d != M * dsub:
        raise ValueError(f"queries have d={d}, codebook expects {M * dsub}")
    lut = torch.empty((nq, M, ksub), dtype=torch.float32, device=q.device)
    _call("mivq_adc_lut", _ptr(q), nq, d, M, nbits, _ptr(centroids), metric, _ptr(lut), _stream())
    return lut


# mivq_adc_search flags (include/mivq.h): the product path always passes ADC_AUTO; the others are
# diagnostics (FORCE_EXACT: same results on the fp32 scan) and test hooks (NO_RERUN leaves the
# queries the filter cannot certify NaN)
ADC_AUTO, ADC_FORCE_EXACT, ADC_NO_RERUN, ADC_SMALL_RERUN_GRID = 0, 1, 2, 4


def adc_search(lut: torch.Tensor, codes_u8: torch.Tensor, k: int, nbits: int,
               id_offset: int = 0, flags: int = ADC_AUTO) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (dists f32 (nq, k), ids int32 (nq, k) holding uint32 bit patterns)."""
    _check(lut, "lut", torch.float32, 3)
    _check(codes_u8, "codes", torch.uint8, 2)
    nq, M, ksub = lut.shape
    n = codes_u8.shape[0]
    if codes_u8.shape[1] != M:
        raise ValueError(f"codes have {codes_u8.shape[1]} sub-codes, LUT has M={M}")
    dists = torch.empty((nq, k), dtype=torch.float32, device=lut.device)
    ids = torch.empty((nq, k), dtype=torch.int32, device=lut.device)
    nb = load_library().mivq_adc_search_workspace_bytes(nq, n, M, nbits, k)
    ws = workspace(nb, lut.device)
    _call("mivq_adc_search", _ptr(lut), nq, _ptr(codes_u8), n, M, nbits, k, id_offset, _ptr(ws), ws.numel(),
          _ptr(dists), _ptr(ids), flags, _stream())
    return dists, ids


def flat_search(q: torch.Tensor, x: torch.Tensor, k: int, metric: int = METRIC_L2,
                id_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    _check(q, "q", torch.float32, 2)
    _check(x, "x", torch.float32, 2)
    nq, d = q.shape
    n = x.shape[0]
    if x.shape[1] != d:
        raise ValueError(f"database has d={x.shape[1]}, queries d={d}")
    dists = torch.empty((nq, k), dtype=torch.float32, device=q.device)
    ids = torch.empty((nq, k), dtype=torch.int32, device=q.device)
    nb = load_library().mivq_flat_search_workspace_bytes(nq, n, d, k)
    ws = workspace(nb, q.device)
    _call("mivq_flat_search", _ptr(q), nq, _ptr(x), n, d, metric, k, id_offset, _ptr(ws), ws.numel(),
          _ptr(dists), _ptr(ids), _stream())
    return dists, ids


def topk_merge(dists: torch.Tensor, ids: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(parts, nq, k) sorted lists -> (nq, k) sorted list, same (dist, id) order."""
    _check(dists, "dists", torch.float32, 3)
    _check(ids, "ids", torch.int32, 3)
    parts, nq, kk = dists.shape
    if kk != k:
        raise ValueError("list length != k")
    od = torch.empty((nq, k), dtype=torch.float32, device=dists.device)
    oi = torch.empty((nq, k), dtype=torch.int32, device=dists.device)
    _call("mivq_topk_merge", _ptr(dists), _ptr(ids), parts, nq, k, _ptr(od), _ptr(oi), _stream())
    return od, oi


# ----------------------------------------------------------------- IVF
def pairwise_distances(x: torch.Tensor, y: torch.Tensor, metric: int = METRIC_L2,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(n, m) exact chains: L2 sum (x-y)^2, IP -(x . y)."""
    _check(x, "x", torch.float32, 2)
    _check(y, "y", torch.float32, 2)
    n, d = x.shape
    m = y.shape[0]
    if y.shape[1] != d:
        raise ValueError(f"pairwise_distances: d mismatch {d} vs {y.shape[1]}")
    if out is None:
        out = torch.empty((n, m), dtype=torch.float32, device=x.device)
    else:
        _check(out, "out", torch.float32, 2)
        if tuple(out.shape) != (n, m):
            raise ValueError("pairwise_distances: out has the wrong shape")
    _call("mivq_pairwise_distances", _ptr(x), n, _ptr(y), m, d, metric, _ptr(out), _stream())
    return out


def topk_rows(dist: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per row the k smallest (value, column); ids int32 holding uint32 bit patterns."""
    _check(dist, "dist", torch.float32, 2)
    n, m = dist.shape
    od = torch.empty((n, k), dtype=torch.float32, device=dist.device)
    oi = torch.empty((n, k), dtype=torch.int32, device=dist.device)
    _call("mivq_topk_rows", _ptr(dist), n, m, k, _ptr(od), _ptr(oi), _stream())
    return od, oi


def bucket_sort(assign: torch.Tensor, K: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Stable bucket sort of (n,) int32 assignments: (offsets int64 (K+1), order int32 (n))."""
    _check(assign, "assign", torch.int32, 1)
    n = assign.shape[0]
    offsets = torch.empty(K + 1, dtype=torch.int64, device=assign.device)
    order = torch.empty(n, dtype=torch.int32, device=assign.device)
    nb = load_library().mivq_bucket_sort_workspace_bytes(n, K)
    ws = workspace(nb, assign.device)
    _call("mivq_bucket_sort", _ptr(assign), n, K, _ptr(offsets), _ptr(order), _ptr(ws), ws.numel(), _stream())
    return offsets, order


def centroid_update(x: torch.Tensor, offsets: torch.Tensor, order: torch.Tensor, centroids: torch.Tensor,
                    counts: torch.Tensor) -> None:
    _check(x, "x", torch.float32, 2)
    _check(offsets, "offsets", torch.int64, 1)
    _check(order, "order", torch.int32, 1)
    _check(centroids, "centroids", torch.float32, 2)
    _check(counts, "counts", torch.int32, 1)
    n, d = x.shape
    K = centroids.shape[0]
    if centroids.shape[1] != d or offsets.shape[0] != K + 1 or counts.shape[0] != K or order.shape[0] != n:
        raise ValueError("centroid_update: shape mismatch")
    _call("mivq_centroid_update", _ptr(x), n, d, K, _ptr(offsets), _ptr(order), _ptr(centroids), _ptr(counts),
          _stream())


def ivf_residuals(x: torch.Tensor, coarse: torch.Tensor, assign: torch.Tensor,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _check(x, "x", torch.float32, 2)
    _check(coarse, "coarse", torch.float32, 2)
    _check(assign, "assign", torch.int32, 1)
    n, d = x.shape
    if coarse.shape[1] != d or assign.shape[0] != n:
        raise ValueError("ivf_residuals: shape mismatch")
    r = torch.empty_like(x) if out is None else out
    _call("mivq_ivf_residuals", _ptr(x), n, d, _ptr(coarse), _ptr(assign), _ptr(r), _stream())
    return r


def gather_rows(src: torch.Tensor, order: torch.Tensor) -> torch.Tensor:
    """dst[i] = src[order[i]] for a contiguous (n, ...) tensor whose rows are 4-byte multiples."""
    _check(order, "order", torch.int32, 1)
    if not src.is_cuda or not src.is_contiguous():
        raise ValueError("gather_rows: src must be a contiguous device tensor")
    row_bytes = src[0].numel() * src.element_size() if src.shape[0] else src.element_size()
    dst = torch.empty((order.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    _call("mivq_gather_rows", _ptr(src), row_bytes, _ptr(order), order.shape[0], _ptr(dst), _stream())
    return dst


def ivfpq_terms(codes_u8: torch.Tensor, pq_centroids: torch.Tensor, prep: torch.Tensor, coarse: torch.Tensor,
                assign: torch.Tensor, nbits: int) -> torch.Tensor:
    _check(codes_u8, "codes", torch.uint8, 2)
    _check(pq_centroids, "pq_centroids", torch.float32, 3)
    _check(coarse, "coarse", torch.float32, 2)
    _check(assign, "assign", torch.int32, 1)
    n, M = codes_u8.shape
    d = coarse.shape[1]
    tau = torch.empty(n, dtype=torch.float32, device=codes_u8.device)
    _call("mivq_ivfpq_terms", _ptr(codes_u8), n, d, M, nbits, _ptr(pq_centroids), _ptr(prep), _ptr(coarse),
          _ptr(assign), _ptr(tau), _stream())
    return tau


def ivfpq_search(lut: torch.Tensor, probe_d: torch.Tensor, probe_l: torch.Tensor, offsets: torch.Tensor,
                 list_codes: torch.Tensor, list_ids: torch.Tensor, tau: Optional[torch.Tensor], metric: int,
                 k: int, nbits: int) -> Tuple[torch.Tensor, torch.Tensor]:
    _check(lut, "lut", torch.float32, 3)
    _check(probe_d, "probe_d", torch.float32, 2)
    _check(probe_l, "probe_l", torch.int32, 2)
    _check(offsets, "offsets", torch.int64, 1)
    _check(list_codes, "list_codes", torch.uint8, 2)
    _check(list_ids, "list_ids", torch.int32, 1)
    if tau is not None:
        _check(tau, "tau", torch.float32, 1)
    nq, M, _ = lut.shape
    nprobe = probe_l.shape[1]
    nlist = offsets.shape[0] - 1
    dists = torch.empty((nq, k), dtype=torch.float32, device=lut.device)
    ids = torch.empty((nq, k), dtype=torch.int32, device=lut.device)
    nb = load_library().mivq_ivfpq_search_workspace_bytes(nq, nprobe, k)
    ws = workspace(nb, lut.device)
    _call("mivq_ivfpq_search", _ptr(lut), nq, M, nbits, _ptr(probe_d), _ptr(probe_l), nprobe, nlist, _ptr(offsets),
          _ptr(list_codes), _ptr(list_ids), _ptr(tau), metric, k, _ptr(ws), ws.numel(), _ptr(dists), _ptr(ids),
          _stream())
    return dists, ids

