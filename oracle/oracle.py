"""CPU parity oracle for the MI355X hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  The product path (``haag_vq`` + ``libmivq.so``) never does.

Functions are numpy-in / numpy-out restatements of the reference algorithms:

* PQ / ADC: ctypes calls into ``oracle/build/liboracle.so`` (mivq_oracle.c), the
  canonical arithmetic defined there (PARITY UNPINNED against faiss, which is absent;
  cross-checked against fp64 brute force on non-near-tie cases).
* SQ: mirrors ``ScalarQuantizer`` (/root/reference/src/haag_vq/methods/
  scalar_quantization.py:37-90) — pinned by tests/golden fixtures generated from the
  reference itself plus the logged KAT (logs/benchmark_runs.db row 38).
* RaBitQ-1: restates faiss ``RaBitQuantizer`` as called by rabit_quantization.py:20-29 —
  pinned by KAT rows 52/53.
* Extended RaBitQ: mirrors ``ExtendedRaBitQuantizer`` (extended_rabitq.py:6-199) —
  pinned by golden fixtures generated from the reference.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "build" / "liboracle.so"
_lib = None


def build() -> Path:
    """Compile liboracle.so (gcc) if it is missing or stale."""
    src = _HERE / "mivq_oracle.c"
    if not _LIB_PATH.exists() or _LIB_PATH.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(str(_LIB_PATH))
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


# ----------------------------------------------------------------------------- PQ
def pq_norms(C: np.ndarray) -> np.ndarray:
    """Canonical ||c_k||^2 (sequential fmaf chain).  C: (M, ksub, dsub) f32."""
    C = np.ascontiguousarray(C, dtype=np.float32)
    M, ksub, dsub = C.shape
    cn = np.empty((M, ksub), np.float32)
    lib().oracle_pq_norms(_p(C), _i32(M), _i32(ksub), _i32(dsub), _p(cn))
    return cn


def pq_encode(X: np.ndarray, C: np.ndarray) -> np.ndarray:
    """Canonical PQ codes, one byte per subspace: (n, M) u8."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    C = np.ascontiguousarray(C, dtype=np.float32)
    M, ksub, dsub = C.shape
    n, d = X.shape
    assert d == M * dsub
    cn = pq_norms(C)
    codes = np.empty((n, M), np.uint8)
    lib().oracle_pq_encode(_p(X), _i64(n), _i32(d), _i32(M), _i32(ksub), _p(C), _p(cn), _p(codes))
    return codes


def pq_scores(xs: np.ndarray, Cm: np.ndarray) -> np.ndarray:
    """All canonical scores of one subvector against one subspace codebook (ksub,)."""
    xs = np.ascontiguousarray(xs, dtype=np.float32)
    Cm = np.ascontiguousarray(Cm, dtype=np.float32)
    ksub, dsub = Cm.shape
    cn = pq_norms(Cm[None])[0]
    out = np.empty(ksub, np.float32)
    lib().oracle_pq_scores(_p(xs), _i32(dsub), _i32(ksub), _p(Cm), _p(cn), _p(out))
    return out


def pq_pack(u8: np.ndarray, nbits: int) -> np.ndarray:
    u8 = np.ascontiguousarray(u8, dtype=np.uint8)
    n, M = u8.shape
    out = np.empty((n, (M * nbits + 7) // 8), np.uint8)
    lib().oracle_pq_pack(_p(u8), _i64(n), _i32(M), _i32(nbits), _p(out))
    return out


def pq_unpack(packed: np.ndarray, M: int, nbits: int) -> np.ndarray:
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    n = packed.shape[0]
    out = np.empty((n, M), np.uint8)
    lib().oracle_pq_unpack(_p(packed), _i64(n), _i32(M), _i32(nbits), _p(out))
    return out


def pq_decode(u8: np.ndarray, C: np.ndarray) -> np.ndarray:
    u8 = np.ascontiguousarray(u8, dtype=np.uint8)
    C = np.ascontiguousarray(C, dtype=np.float32)
    M, ksub, dsub = C.shape
    n = u8.shape[0]
    out = np.empty((n, M * dsub), np.float32)
    lib().oracle_pq_decode(_p(u8), _i64(n), _i32(M * dsub), _i32(M), _i32(ksub), _p(C), _p(out))
    return out


def pq_encode_fp64(X: np.ndarray, C: np.ndarray):
    """fp64 brute-force nearest centroid + the relative top-2 gap per (row, subspace).

    Independent of the canonical fp32 order: any correct implementation must agree with
    it wherever the gap exceeds the fp32 rounding bound.
    """
    X = np.asarray(X, np.float64)
    C = np.asarray(C, np.float64)
    M, ksub, dsub = C.shape
    n = X.shape[0]
    Xs = X.reshape(n, M, dsub)
    codes = np.empty((n, M), np.uint8)
    gap = np.empty((n, M), np.float64)
    for m in range(M):
        # |x|^2 + |c|^2 - 2 x.c in fp64 (BLAS): its rounding (~1e-15 of the scale) is far
        # below any gap this is used to certify (>= 1e-5 of the scale)
        xx = (Xs[:, m] ** 2).sum(-1)
        cc = (C[m] ** 2).sum(-1)
        dist = xx[:, None] + cc[None, :] - 2.0 * (Xs[:, m] @ C[m].T)  # (n, ksub)
        if ksub > 1:
            top2 = np.argpartition(dist, 1, axis=1)[:, :2]
            d2 = np.take_along_axis(dist, top2, 1)
            first = np.where(d2[:, 0] <= d2[:, 1], 0, 1)
            codes[:, m] = top2[np.arange(n), first]
            d0 = d2[np.arange(n), first]
            d1 = d2[np.arange(n), 1 - first]
            scale = xx + cc.max()
            gap[:, m] = (d1 - d0) / np.maximum(scale, 1e-300)
        else:
            codes[:, m] = 0
            gap[:, m] = np.inf
    return codes, gap


# ----------------------------------------------------------------------------- ADC
def adc_lut(Q: np.ndarray, C: np.ndarray, metric: int = 1) -> np.ndarray:
    """metric 1 = L2 (squared distances), 0 = inner product (stored negated)."""
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    C = np.ascontiguousarray(C, dtype=np.float32)
    M, ksub, dsub = C.shape
    nq = Q.shape[0]
    lut = np.empty((nq, M, ksub), np.float32)
    lib().oracle_adc_lut(_p(Q), _i64(nq), _i32(M * dsub), _i32(M), _i32(ksub), _p(C), _i32(metric), _p(lut))
    return lut


def flat_search(Q: np.ndarray, X: np.ndarray, k: int, metric: int = 1, id_offset: int = 0):
    """Exact top-k (dist, id); IP distances are negated inner products (ascending)."""
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    X = np.ascontiguousarray(X, dtype=np.float32)
    nq, d = Q.shape
    n = X.shape[0]
    dists = np.empty((nq, k), np.float32)
    ids = np.empty((nq, k), np.uint32)
    lib().oracle_flat_search(_p(Q), _i64(nq), _p(X), _i64(n), _i32(d), _i32(metric), _i32(k), _i64(id_offset),
                             _p(dists), _p(ids))
    return dists, ids


def adc_search(lut: np.ndarray, codes_u8: np.ndarray, k: int, id_offset: int = 0):
    lut = np.ascontiguousarray(lut, dtype=np.float32)
    codes_u8 = np.ascontiguousarray(codes_u8, dtype=np.uint8)
    nq, M, ksub = lut.shape
    n = codes_u8.shape[0]
    dists = np.empty((nq, k), np.float32)
    ids = np.empty((nq, k), np.uint32)
    lib().oracle_adc_search(_p(lut), _i64(nq), _p(codes_u8), _i64(n), _i32(M), _i32(ksub),
                            _i32(k), _i64(id_offset), _p(dists), _p(ids))
    return dists, ids


# ----------------------------------------------------------------------------- SQ
def sq_fit(X: np.ndarray):
    """lo, hi, den exactly as scalar_quantization.py:37-39,54 compute them."""
    lo = X.min(axis=0)
    hi = X.max(axis=0)
    den = hi - lo + 1e-8
    return lo, hi, den


def sq_encode(X: np.ndarray, lo: np.ndarray, den: np.ndarray, nbits: int) -> np.ndarray:
    X = np.ascontiguousarray(X)
    n, d = X.shape
    if nbits == 16:
        out = np.empty((n, d), np.uint16)
    elif nbits == 8:
        out = np.empty((n, d), np.uint8)
    else:
        out = np.empty((n, (d + 1) // 2), np.uint8)
    if X.dtype == np.float64:
        lib().oracle_sq_encode_f64(_p(X), _i64(n), _i32(d), _p(np.ascontiguousarray(lo, np.float64)),
                                   _p(np.ascontiguousarray(den, np.float64)), _i32(nbits), _p(out))
    else:
        X = np.ascontiguousarray(X, np.float32)
        lib().oracle_sq_encode_f32(_p(X), _i64(n), _i32(d), _p(np.ascontiguousarray(lo, np.float32)),
                                   _p(np.ascontiguousarray(den, np.float32)), _i32(nbits), _p(out))
    return out


def sq_encode_numpy(X: np.ndarray, lo: np.ndarray, den: np.ndarray, nbits: int = 8) -> np.ndarray:
    """ScalarQuantizer._compress_block (scalar_quantization.py:52-68) as the reference writes it,
    in numpy (the CPU path the reference runs; 8 and 16 bits): ((X - lo) / den * (2^b - 1)),
    rounded half to even, cast to uint8 / uint16.  The bench's CPU baseline for SQ-8."""
    q = np.round((X - lo) / den * float((1 << nbits) - 1))
    return q.astype(np.uint16 if nbits == 16 else np.uint8)


def sq_decode(codes: np.ndarray, d: int, lo: np.ndarray, den: np.ndarray, nbits: int) -> np.ndarray:
    codes = np.ascontiguousarray(codes)
    n = codes.shape[0]
    if lo.dtype == np.float64:
        out = np.empty((n, d), np.float64)
        lib().oracle_sq_decode_f64(_p(codes), _i64(n), _i32(d), _p(np.ascontiguousarray(lo)),
                                   _p(np.ascontiguousarray(den)), _i32(nbits), _p(out))
    else:
        out = np.empty((n, d), np.float32)
        lib().oracle_sq_decode_f32(_p(codes), _i64(n), _i32(d), _p(np.ascontiguousarray(lo, np.float32)),
                                   _p(np.ascontiguousarray(den, np.float32)), _i32(nbits), _p(out))
    return out


# ----------------------------------------------------------------------------- RaBitQ-1
def rabitq_encode(X: np.ndarray, centroid=None, metric: int = 1) -> np.ndarray:
    X = np.ascontiguousarray(X, np.float32)
    n, d = X.shape
    codes = np.empty((n, (d + 7) // 8 + 8), np.uint8)
    c = None if centroid is None else np.ascontiguousarray(centroid, np.float32)
    lib().oracle_rabitq_encode(_p(X), _i64(n), _i32(d), None if c is None else _p(c), _i32(metric), _p(codes))
    return codes


def rabitq_decode(codes: np.ndarray, d: int, centroid=None) -> np.ndarray:
    codes = np.ascontiguousarray(codes, np.uint8)
    n = codes.shape[0]
    out = np.empty((n, d), np.float32)
    c = None if centroid is None else np.ascontiguousarray(centroid, np.float32)
    lib().oracle_rabitq_decode(_p(codes), _i64(n), _i32(d), None if c is None else _p(c), _p(out))
    return out


# ----------------------------------------------------------------------------- Extended RaBitQ
def rabitq_est(codes: np.ndarray, d: int, Q: np.ndarray, centroid=None, qb: int = 4, metric: int = 1) -> np.ndarray:
    """RaBitQ estimator keys (nq, n) of IndexRaBitQ search (see oracle_rabitq_est); ascending ranks best."""
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    c = None if centroid is None else np.ascontiguousarray(centroid, dtype=np.float32)
    nq, n = Q.shape[0], codes.shape[0]
    out = np.empty((nq, n), np.float32)
    lib().oracle_rabitq_est(_p(codes), _i64(n), _i32(d), _p(Q), _i64(nq), None if c is None else _p(c),
                            _i32(qb), _i32(metric), _p(out))
    return out


def lloyd_1d_normal(num_levels: int, seed: int, n_samples: int = 200_000,
                    max_iter: int = 100, tol: float = 1e-7) -> np.ndarray:
    """Restates extended_rabitq.py:6-44 (1-D Lloyd on an N(0,1) sample)."""
    rng = np.random.default_rng(seed)
    samples = rng.standard_normal(n_samples)
    levels = np.quantile(samples, (np.arange(num_levels) + 0.5) / num_levels)
    for _ in range(max_iter):
        idx = np.searchsorted(0.5 * (levels[:-1] + levels[1:]), samples)
        new = levels.copy()
        for k in range(num_levels):
            sel = idx == k
            if np.any(sel):
                new[k] = samples[sel].mean()
        new.sort()
        shift = float(np.max(np.abs(new - levels)))
        levels = new
        if shift < tol:
            break
    return levels.astype(np.float64)


def extrabitq_fit(X: np.ndarray, num_bits: int, seed: int = 0):
    """Model state of extended_rabitq.py:90-106: centroid, QR rotation, Lloyd levels."""
    X = np.asarray(X)
    D = X.shape[1]
    c = X.mean(axis=0).astype(np.float64)
    P, _ = np.linalg.qr(np.random.default_rng(seed).standard_normal((D, D)))
    return c, P.astype(np.float64), lloyd_1d_normal(2 ** num_bits, seed=seed)


def extrabitq_encode(X, c, P, levels, num_bits, eps=1e-12) -> np.ndarray:
    """Restates extended_rabitq.py:125-170 (fp64; MSB-first index packing)."""
    X = np.asarray(X, np.float64)
    N, D = X.shape
    r = X - c
    nrm = np.linalg.norm(r, axis=1)
    o = r / np.maximum(nrm, eps)[:, None]
    s = (o @ P) * np.sqrt(D)
    idx = np.searchsorted(0.5 * (levels[:-1] + levels[1:]), s).astype(np.int64)
    sh = levels[idx]
    num = np.einsum("nd,nd->n", s, sh)
    den = np.einsum("nd,nd->n", sh, sh)
    t = np.where(den > eps, num / den, 1.0)
    ib = (D * num_bits + 7) // 8
    out = np.zeros((N, ib + 8), np.uint8)
    bits = ((idx[:, :, None] >> np.arange(num_bits - 1, -1, -1)) & 1).astype(np.uint8)
    out[:, :ib] = np.packbits(bits.reshape(N, D * num_bits), axis=1)
    out[:, ib:ib + 4] = nrm.astype(np.float32).view(np.uint8).reshape(N, 4)
    out[:, ib + 4:ib + 8] = t.astype(np.float32).view(np.uint8).reshape(N, 4)
    return out


def extrabitq_decode(codes, c, P, levels, num_bits) -> np.ndarray:
    """Restates extended_rabitq.py:173-198."""
    codes = np.ascontiguousarray(codes, np.uint8)
    N = codes.shape[0]
    D = P.shape[0]
    ib = (D * num_bits + 7) // 8
    bits = np.unpackbits(codes[:, :ib], axis=1)[:, :D * num_bits].reshape(N, D, num_bits).astype(np.int64)
    idx = bits @ (1 << np.arange(num_bits - 1, -1, -1)).astype(np.int64)
    sh = levels[idx]
    nrm = codes[:, ib:ib + 4].copy().view(np.float32).reshape(N).astype(np.float64)
    t = codes[:, ib + 4:ib + 8].copy().view(np.float32).reshape(N).astype(np.float64)
    return ((((sh / np.sqrt(D)) * t[:, None]) @ P.T) * nrm[:, None] + c).astype(np.float32)


# ----------------------------------------------------------------------------- IVF / IVF-PQ
# Restates FaissIvfPqIndex (methods/search/faiss_ivfpq_index.py:46-76; faiss IndexIVFPQ,
# by_residual) with the canonical arithmetic of include/mivq.h.  PARITY UNPINNED (faiss absent).
def pairwise(X: np.ndarray, Y: np.ndarray, metric: int = 1) -> np.ndarray:
    X = np.ascontiguousarray(X, dtype=np.float32)
    Y = np.ascontiguousarray(Y, dtype=np.float32)
    out = np.empty((X.shape[0], Y.shape[0]), np.float32)
    lib().oracle_pairwise(_p(X), _i64(X.shape[0]), _p(Y), _i64(Y.shape[0]), _i32(X.shape[1]), _i32(metric), _p(out))
    return out


def topk_rows(D: np.ndarray, k: int):
    """Per row the k smallest (value, column) pairs; NaN ranks as +inf; pads (+inf, NO_ID)."""
    D = np.asarray(D, np.float32)
    n, m = D.shape
    key = np.where(np.isnan(D), np.inf, D)
    order = np.lexsort((np.broadcast_to(np.arange(m), (n, m)), key), axis=1)[:, :k]
    dd = np.full((n, k), np.inf, np.float32)
    ii = np.full((n, k), 0xFFFFFFFF, np.uint32)
    kk = order.shape[1]
    dd[:, :kk] = np.take_along_axis(key, order, 1)
    ii[:, :kk] = order.astype(np.uint32)
    return dd, ii


def bucket_sort(assign: np.ndarray, K: int):
    """(offsets (K+1) int64, order) — rows of each bucket in ascending row order."""
    assign = np.asarray(assign, np.int64)
    order = np.argsort(assign, kind="stable").astype(np.uint32)
    offsets = np.zeros(K + 1, np.int64)
    offsets[1:] = np.cumsum(np.bincount(assign, minlength=K))
    return offsets, order


def centroid_update(X: np.ndarray, assign: np.ndarray, C: np.ndarray):
    X = np.ascontiguousarray(X, dtype=np.float32)
    C = np.array(C, dtype=np.float32, copy=True)
    K, d = C.shape
    a = np.ascontiguousarray(assign, dtype=np.uint32)
    counts = np.empty(K, np.int32)
    lib().oracle_centroid_update(_p(X), _i64(X.shape[0]), _i32(d), _i32(K), _p(a), _p(C), _p(counts))
    return C, counts


def ivfpq_terms(codes_u8: np.ndarray, Cpq: np.ndarray, coarse: np.ndarray, assign: np.ndarray) -> np.ndarray:
    codes_u8 = np.ascontiguousarray(codes_u8, dtype=np.uint8)
    Cpq = np.ascontiguousarray(Cpq, dtype=np.float32)
    coarse = np.ascontiguousarray(coarse, dtype=np.float32)
    a = np.ascontiguousarray(assign, dtype=np.uint32)
    M, ksub, dsub = Cpq.shape
    cn = pq_norms(Cpq)
    n = codes_u8.shape[0]
    tau = np.empty(n, np.float32)
    lib().oracle_ivfpq_terms(_p(codes_u8), _i64(n), _i32(M * dsub), _i32(M), _i32(ksub), _p(Cpq), _p(cn),
                             _p(coarse), _p(a), _p(tau))
    return tau


def ivfpq_search(lut, probe_d, probe_l, offsets, list_codes, list_ids, tau, metric: int, k: int):
    lut = np.ascontiguousarray(lut, dtype=np.float32)
    nq, M, ksub = lut.shape
    probe_d = np.ascontiguousarray(probe_d, dtype=np.float32)
    probe_l = np.ascontiguousarray(probe_l, dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    list_codes = np.ascontiguousarray(list_codes, dtype=np.uint8)
    list_ids = np.ascontiguousarray(list_ids, dtype=np.uint32)
    tau = np.ascontiguousarray(tau if tau is not None else np.zeros(list_ids.shape[0]), dtype=np.float32)
    dists = np.empty((nq, k), np.float32)
    ids = np.empty((nq, k), np.uint32)
    lib().oracle_ivfpq_search(_p(lut), _i64(nq), _i32(M), _i32(ksub), _p(probe_d), _p(probe_l),
                              _i32(probe_l.shape[1]), _p(offsets), _p(list_codes), _p(list_ids), _p(tau),
                              _i32(metric), _i32(k), _p(dists), _p(ids))
    return dists, ids


def ivfpq_build(X: np.ndarray, coarse: np.ndarray, Cpq: np.ndarray, metric: int = 1):
    """Full IVF-PQ add of X: (assign, codes, offsets, list_codes, list_ids, tau-in-list-order)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    coarse = np.ascontiguousarray(coarse, dtype=np.float32)
    K = coarse.shape[0]
    _, a = topk_rows(pairwise(X, coarse, metric), 1)
    a = a[:, 0]
    R = (X - coarse[a.astype(np.int64)]).astype(np.float32)
    codes = pq_encode(R, Cpq)
    tau = ivfpq_terms(codes, Cpq, coarse, a) if metric == 1 else np.zeros(X.shape[0], np.float32)
    offsets, order = bucket_sort(a, K)
    return a, codes, offsets, codes[order], order, tau[order]


def ivfpq_query(Q: np.ndarray, coarse: np.ndarray, Cpq: np.ndarray, built, nprobe: int, k: int, metric: int = 1):
    _, _, offsets, list_codes, list_ids, tau = built
    pd, pl = topk_rows(pairwise(Q, coarse, metric), nprobe)
    lut = adc_lut(Q, Cpq, 0)
    return ivfpq_search(lut, pd, pl, offsets, list_codes, list_ids, tau if metric == 1 else None, metric, k)


# ----------------------------------------------------------------------------- metrics
def exact_l2_topk(Q: np.ndarray, X: np.ndarray, k: int) -> np.ndarray:
    """Exact L2 top-k ids (fp64 distances, stable ties by id) — ground-truth helper."""
    Q = np.asarray(Q, np.float64)
    X = np.asarray(X, np.float64)
    d = (Q ** 2).sum(1)[:, None] + (X ** 2).sum(1)[None, :] - 2.0 * Q @ X.T
    return np.argsort(d, axis=1, kind="stable")[:, :k]


def cpu_threads() -> int:
    """Threads the OpenMP oracle actually runs with (OMP_NUM_THREADS, else the affinity mask)."""
    env = os.environ.get("OMP_NUM_THREADS", "").split(",")[0].strip()
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1
