"""Benchmark: PQ-encode vectors/s (+ ADC queries/s @ recall@10) on synthetic N x 1536 fp32.

Headline (BASELINE.json configs[1]): PQ M=16 B=8 encode of 1M x 1536 fp32 per
GPU, rows = unit-normalised Gaussian (`--data gaussian`, the §8d distribution), generated on
the device from seed = rank (weak scaling: every rank owns its own shard).  One "step" = one
`mivq_pq_encode` call over the resident shard (fp16-MFMA filter kernel, exact re-check
kernels, code transpose).  Codebooks: rank 0 trains them on its first 65,536 rows (GPU
k-means, 25 iterations, seed 1234) and broadcasts them (RCCL).

Second-level legs (keys of the same JSON line):
  adc        ADC top-10 of --nq queries (the first rows of rank 0's shard, the reference's
             convention) over all shards (queries broadcast, per-shard LUT
             scan, one RCCL all-gather, on-device merge): queries/s, recall@10 against the
             exact top-10 over the raw vectors, recall@10 and top-10 agreement of the
             reference's own search on the same codes (decode + exact L2), the LDS roofline
             of the scan, and (rank 0, N = 1) the oracle's ADC on the host cores.
  alt_data   the headline encode on the other synthetic distribution (clustered rows).
  north_star (N = 1 only) the north-star size: the headline encode on 10M x 1536 Gaussian
             rows (BASELINE north_star "10M x 1536 at 1 GPU"), parity on a 200,000-row sample.
  config5    BASELINE configs[4], the MS MARCO shape: 6.65M x 1024 rows per GPU (53.2M over
             8 GPUs), PQ16 encode + ADC top-10 of 10,000 queries with the RCCL merge.
  configs    (N = 1 only) the sweep's PQ8 shape at 1M x 1536 (dsub 192, BASELINE configs[0]),
             configs[2] OPQ32 encode + ADC recall@10 (1M x 1536) and configs[3]
             SQ-8 / RaBitQ-1 encode + search (1M x 3072), each with its own roofline, and the
             registry's `rabitq` route (Extended RaBitQ, 4 bits, 200k x 3072 encode + decode,
             fp64 MFMA roofline of erq_rotate_kernel).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
  --gpus N > 1 without WORLD_SIZE in the environment starts
  `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child process (no
  exec; nothing here touches the GPU before that) and exits with its status; rank 0 prints
  the JSON line.  Under torch.distributed.run (WORLD_SIZE set) --gpus must equal WORLD_SIZE.
  --dry-run: no GPU: the same launcher and rank plumbing over gloo on CPU tensors (codebook
  and query broadcast, per-shard exact top-k in torch, all-gather + merge), checked against
  the single-rank result — a harness test, not a measurement.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))

from haag_vq import _native  # noqa: E402  (loads nothing and touches no GPU at import)
from haag_vq.parallel import sharded  # noqa: E402

METRIC = "PQ-encode vectors/sec + ADC queries/sec @ recall@10, 1M×1536 fp32"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
SETTLE_MS = 60.0               # untimed busy time after the W warmup calls of an encode leg (timed())
MFMA_F32_PEAK_TFS = 157.3      # dense fp32 matrix peak (same table)
MFMA_F16_PEAK_TFS = 2516.6     # dense f16/bf16 matrix peak = 16 x fp32 (same table)
MFMA_F64_PEAK_TFS = 78.6       # dense fp64 matrix peak (MI355X spec; not in the guide's table)
INT8_MFMA_PEAK_TOPS = 2 * MFMA_F16_PEAK_TFS  # v_mfma_i32_32x32x32_i8: the cycles of the f16 32x32x16 at 2x K
LDS_PEAK_GBS = 256 * 256 * 2.4  # 256 CUs x 256 B/clk (ds_read_b128) x 2.4 GHz = 157 TB/s
# The filtered ADC scan (adc_qscan_kernel) is VALU-issue bound (its LDS reads are
# conflict-free since round 6 and PMC shows the VALU pipe saturated, profiles/r06_s1/pmc_*).
# Its roofline is the chip's VALU issue rate for its instruction mix: the static count of one
# wave-step (64 rows x 16 queries) of the built kernel, split by encoding (tools/isa_qscan.py,
# checked against the library by tests/test_abi.py) ...
QSCAN_VALU_PER_STEP = {16: {"valu_32bit": 64, "valu_64bit": 106}, 32: {"valu_32bit": 99, "valu_64bit": 187}}
# ... priced at the issue rates tools/probes/valu_rate.hip measured with 4 waves per SIMD on every
# CU (chip wave-instructions/s under that load; profiles/r06_s5/valu_rate.log): 32-bit-encoded
# VALU (v_add_u32_e32) 0.881e12, 64-bit-encoded VALU (v_perm_b32 / v_med3_u32 / v_lshl_or_b32,
# all equal) 0.577e12
VALU_RATE_32BIT = 0.881e12
VALU_RATE_64BIT = 0.577e12


def qscan_valu_roofline(nq, n, M, seconds):
    """VALU issue roofline of the integer scan: achieved = its VALU wave-instructions (static count
    per wave-step x wave-steps) / the timed search; peak = the mix-weighted probe rate.  The timed
    region is the whole mivq_adc_search (table prep, rerank, re-run included), so this is a lower
    bound of the scan's own rate."""
    v = QSCAN_VALU_PER_STEP.get(M)
    if v is None:
        return None
    steps = -(-nq // 16) * (n / 64.0)  # wave-steps: query blocks x 64-row groups
    instr = steps * (v["valu_32bit"] + v["valu_64bit"])
    peak = (v["valu_32bit"] + v["valu_64bit"]) / (v["valu_32bit"] / VALU_RATE_32BIT + v["valu_64bit"] / VALU_RATE_64BIT)
    return {"achieved": instr / seconds / 1e9, "peak": peak / 1e9, "unit": "G VALU wave-instructions/s",
            "frac": instr / seconds / peak, "valu_per_wave_step": v,
            "valu_instructions_per_search": instr}
# rigorous relative bound on a canonical fp32 score difference (oracle header): 2 (2 g_96 + u)
CLEAR_GAP = 3e-5


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=1_000_000, help="rows per GPU")
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--nq", type=int, default=1000, help="ADC queries")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--gt-queries", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    ap.add_argument("--data", choices=("gaussian", "clustered"), default="gaussian")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-adc", action="store_true")
    ap.add_argument("--no-alt-data", action="store_true")
    ap.add_argument("--no-north-star", action="store_true")
    ap.add_argument("--north-star-rows", type=int, default=10_000_000)
    ap.add_argument("--no-config5", action="store_true")
    ap.add_argument("--no-configs", action="store_true")
    ap.add_argument("--config5-rows", type=int, default=6_650_000, help="config #5 rows per GPU")
    ap.add_argument("--config5-nq", type=int, default=10_000)
    ap.add_argument("--opq-iters", type=int, default=4)
    ap.add_argument("--erq-rows", type=int, default=200_000, help="Extended RaBitQ leg rows (D = 3072)")
    ap.add_argument("--exact", action="store_true", help="force the exact VALU encode path")
    ap.add_argument("--legacy", action="store_true", help="diagnostic: subspace-looping MFMA kernel")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo rehearsal of the rank plumbing")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(a) -> int:
    """One process per GPU under torch.distributed.run, started as a child (never exec'd)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           # "--": torchrun's parser would take bench flags that abbreviate its own options
           # (--n, --d) as ambiguous options of its own
           "--", str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"[launcher] {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------- data
def synth(n, d, seed, dev, kind="gaussian", centers_seed=12345, n_centers=4096, spread=0.02):
    """Synthetic embedding-like rows, generated on the device.

    gaussian : isotropic N(0, I) rows, L2-normalised (no neighbourhood structure,
               so recall@k of any quantizer is low on it; the hardest case for the filter).
    clustered: normalise(center[j] + spread * N(0, I)) with 4096 shared unit centers (seeded
               identically on every rank) — neighbourhoods like real text embeddings.
    """
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    step = 1 << 20
    if kind == "gaussian":
        X = torch.randn((n, d), generator=g, device=dev, dtype=torch.float32)
    else:
        gc = torch.Generator(device=dev)
        gc.manual_seed(centers_seed)
        cen = torch.randn((n_centers, d), generator=gc, device=dev, dtype=torch.float32)
        cen /= torch.linalg.vector_norm(cen, dim=1, keepdim=True)
        X = torch.empty((n, d), device=dev, dtype=torch.float32)
        for s in range(0, n, step):
            e = min(n, s + step)
            a = torch.randint(0, n_centers, (e - s,), generator=g, device=dev)
            X[s:e] = cen[a] + spread * torch.randn((e - s, d), generator=g, device=dev, dtype=torch.float32)
    for s in range(0, n, step):  # in place, in slices (no second copy of a 27 GB shard)
        X[s:s + step] /= torch.linalg.vector_norm(X[s:s + step], dim=1, keepdim=True)
    return X


def traffic_from_profile(workload: str):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (profiles/traffic.json,
    written by tools/traffic.py), if it is for this workload AND was measured on this build:
    the entry's kernel-source hash must equal _native.kernel_source_hash() of the running tree
    (a stale entry gives None, never a number from other kernels)."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        e = json.loads(p.read_text()).get(workload, {})
    except Exception:
        return None
    if e.get("kernel_source_hash") != _native.kernel_source_hash():
        return None
    return e.get("bytes_per_launch")


SETTLE = {"extra_steps": 0}


def timed(fn, steps, warmup, world=1, dev=None, settle_ms=0.0):
    """W untimed calls; K timed calls bracketed by barrier + synchronize; HIP events on the
    current stream (the one libmivq launches on) around every call.  Returns (wall s/step
    max over ranks, device ms/call mean).

    settle_ms > 0: after the W warmup calls, further untimed calls until the warm-up has kept
    the GPU busy for settle_ms.  The MI355X's power management needs ~30 ms of continuous load
    to settle: in kernel traces of back-to-back 1M-row encodes the filter launches average
    1.35-1.37 ms over calls 1-10, 1.22 ms over calls 11-20 and 1.17-1.18 ms after that
    (profiles/r02_s10_power_transient.txt); timing K = 20 calls after W = 5 would average
    that transient into a steady-state throughput figure.  The count of extra calls is
    reported (SETTLE)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if settle_ms > 0:
        t0 = time.perf_counter()
        extra = 0
        while (time.perf_counter() - t0) * 1e3 < settle_ms:
            fn()
            torch.cuda.synchronize()
            extra += 1
        SETTLE["extra_steps"] = max(SETTLE["extra_steps"], extra)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt / steps, float(np.mean([s.elapsed_time(e) for s, e in evs]))


def _oracle():
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O  # CPU restatement: baseline legs and live parity checks only

    return O


# ------------------------------------------------------------------------- PQ encode
def train_codebook(X, M, nbits, rank, world, dev):
    from haag_vq.methods._kmeans import train_pq

    C = torch.empty((M, 1 << nbits, X.shape[1] // M), dtype=torch.float32, device=dev)
    if rank == 0:
        t0 = time.perf_counter()
        C.copy_(train_pq(X[:65536], M, nbits, niter=25, seed=1234, exact_assign=True))
        torch.cuda.synchronize()
        log(f"[rank 0] k-means fit on 65536 rows: {time.perf_counter() - t0:.2f} s")
    sharded.broadcast_(C)  # replicated codebooks
    return C


def encode_leg(X, C, a, rank, world, dev, steps, warmup, exact=False, legacy=False):
    nbits = 8
    prep = _native.pq_prepare(C, nbits)
    n, d = X.shape
    M = C.shape[0]
    codes = torch.empty((n, _native.pq_code_size(M, nbits)), dtype=torch.uint8, device=dev)
    flags = _native.MIVQ_PQ_LEGACY_MFMA if legacy else 0
    fn = lambda: _native.pq_encode(X, C, prep, nbits, exact=exact, out=codes, flags_extra=flags)  # noqa: E731
    wall, kern_ms = timed(fn, steps, warmup, world, dev, settle_ms=SETTLE_MS)
    bpv = 4 * d + M  # read x, write the codes
    ach = n * bpv / (kern_ms * 1e-3) / 1e9
    return codes, {"wall_s": wall, "kernel_ms": kern_ms, "bytes_per_vector": bpv, "achieved_gbs": ach}


def parity_check(X, C, codes, O, max_rows=None, fp64_rows=20000):
    """GPU codes vs the oracle's canonical encode (bit-exact) on the first rows, and vs an
    fp64 brute-force nearest centroid wherever its top-2 gap clears the fp32 rounding bound."""
    n = X.shape[0] if max_rows is None else min(max_rows, X.shape[0])
    Cn = C.cpu().numpy()
    got = codes[:n].cpu().numpy()
    Xh = X[:n].cpu().numpy()
    t0 = time.perf_counter()
    ref = O.pq_encode(Xh, Cn)
    t_or = time.perf_counter() - t0
    nf = min(fp64_rows, n)
    c64, gap = O.pq_encode_fp64(Xh[:nf], Cn)
    clear = gap > CLEAR_GAP
    return {"rows_checked": n, "mismatched_codes": int((got != ref).sum()),
            "fp64_rows": nf, "fp64_clear_fraction": float(clear.mean()),
            "fp64_clear_mismatches": int((got[:nf][clear] != c64[clear]).sum()),
            "fp64_rule": f"fp64 argmin where the relative top-2 gap > {CLEAR_GAP:g}"}, t_or


def cpu_baseline(X, C, O, target_s):
    """The oracle's PQ encode (OpenMP C restatement) on a bounded sample of the shard."""
    threads = O.cpu_threads()
    Cn = C.cpu().numpy()
    n_cal = 2000
    t0 = time.perf_counter()
    O.pq_encode(X[:n_cal].cpu().numpy(), Cn)
    dt = time.perf_counter() - t0
    n_s = int(min(X.shape[0], max(n_cal, n_cal * target_s / max(dt, 1e-6))))
    Xs = X[:n_s].cpu().numpy()
    t0 = time.perf_counter()
    O.pq_encode(Xs, Cn)
    dt = time.perf_counter() - t0
    return {"value": n_s / dt, "unit": "vectors/s", "cores": threads, "kind": "port",
            "sample": f"first {n_s} rows of rank 0's shard, oracle/mivq_oracle.c pq_encode (OpenMP, AVX2), "
                      f"{dt:.1f} s wall on {threads} threads = {dt * threads:.0f} thread-s"}


# ------------------------------------------------------------------------- ADC
def adc_leg(X, C, codes, a, rank, world, dev, Q, k, gt_queries, reps=30, cpu=True):
    """Sharded ADC search + its roofline + the reference's decode-then-exact ranking on the
    same codes (+ the oracle's ADC on the host cores at N = 1).

    reps: 30 calls of ~0.45 ms at 1000 x 1M (10 calls, a 5 ms timed region, read ~6 % slow: the
    host's first enqueue and the final synchronize are not amortised; tools/probe_adc_wall.py,
    profiles/r06_s37); the 20 ms config #5 calls take 2."""
    nbits = 8
    n, d = X.shape
    M = C.shape[0]
    nq = Q.shape[0]
    sharded.broadcast_(Q)
    off = rank * n
    search = lambda: sharded.sharded_adc_search(Q, C, codes, nbits, k, off)  # noqa: E731
    wall, dev_ms = timed(search, reps, 1, world, dev)
    ad, ai = search()
    # mivq_adc_search alone (no LUT build, no exchange): for M = 16 / 32 the filtered path
    # (integer-LUT scan, exact fp32 re-rank + certificate, fp32 re-run of uncertified queries:
    # DESIGN §3.3), every launch of it inside the timed call
    lut = _native.adc_lut(Q, C, nbits)
    _, scan_ms = timed(lambda: _native.adc_search(lut, codes, k, nbits, id_offset=off), reps, 1)
    gq = min(gt_queries, nq)
    Qg = Q[:gq].contiguous()
    _, gi = sharded.sharded_exact_search(Qg, X, k, off)  # exact top-k over the raw vectors
    Xhat = _native.pq_decode(codes, C, nbits)            # reference search: decode + exact L2
    _, di = sharded.sharded_exact_search(Qg, Xhat, k, off)
    del Xhat
    got = ai[:gq].cpu().numpy().view(np.uint32)
    gt = gi.cpu().numpy().view(np.uint32)
    dec = di.cpu().numpy().view(np.uint32)
    rec = lambda ref, x: float(np.mean([len(set(ref[j]) & set(x[j])) / k for j in range(gq)]))  # noqa: E731
    vr = qscan_valu_roofline(nq, n, M, scan_ms * 1e-3)
    out = {"qps": nq / wall, "nq": nq, "k": k, "n_total": n * world, "ms_per_batch": wall * 1e3,
           f"recall@{k}": rec(gt, got), "recall_queries": gq,
           f"recall@{k}_decode_exact": rec(gt, dec), "topk_agreement_adc_vs_decode_exact": rec(dec, got),
           "gt": "exact L2 top-k over the raw vectors (mivq_flat_search, sharded + merged)",
           "roofline": dict({"bound": "valu", "kernel": "mivq_adc_search (per rank: adc_qstats + adc_qtab + adc_qscan_kernel "
                                                        "+ adc_rerank_kernel + fp32 re-run of uncertified queries)",
                             "scan_ms": scan_ms,
                             # the integer scan's own LDS reads (one byte per (query, row, subspace),
                             # conflict-free since round 6) against the LDS peak, for reference
                             "lds_bytes_read_frac": nq * n * M / (scan_ms * 1e-3) / 1e9 / LDS_PEAK_GBS,
                             "note": "VALU-issue roofline of the integer scan (bench.py qscan_valu_roofline, "
                                     "DESIGN 3.3): static VALU per wave-step of the built kernel priced at the "
                                     "measured issue rates; the timed region is the whole search"},
                            **(vr or {"bound": "lds", "achieved": nq * n * M * 4 / (scan_ms * 1e-3) / 1e9,
                                      "peak": LDS_PEAK_GBS, "unit": "GB/s (fp32 LUT entries, the fp32 scan)",
                                      "frac": nq * n * M * 4 / (scan_ms * 1e-3) / 1e9 / LDS_PEAK_GBS}))}
    if cpu and rank == 0 and world == 1:
        O = _oracle()
        # a bounded sample: ~1 s wall on the box's 16 threads (~16 thread-s)
        nqs = min(nq, 2000)
        Qh, Cn = Q[:nqs].cpu().numpy(), C.cpu().numpy()
        ch = codes.cpu().numpy()
        t0 = time.perf_counter()
        rd, ri = O.adc_search(O.adc_lut(Qh, Cn), ch, k)
        dt = time.perf_counter() - t0
        ok = np.array_equal(ri, ai[:nqs].cpu().numpy().view(np.uint32))
        # oracle_adc_lut / oracle_adc_search are OpenMP loops over queries
        # (oracle/mivq_oracle.c:379,407): the threads that ran are min(OpenMP threads, queries)
        threads = min(O.cpu_threads(), nqs)
        out["cpu_baseline"] = {"value": nqs / dt, "unit": "queries/s", "cores": threads, "kind": "port",
                               "sample": f"{nqs} queries x {n} codes, oracle adc_lut + adc_search "
                                         f"(C, OpenMP over queries, {threads} threads), {dt:.1f} s wall",
                               "ids_equal_gpu": ok}
    return out


# ------------------------------------------------------------------------- other configs
def opq32_leg(a, dev, steps, warmup, cpu=True):
    from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer

    d, M, n = 1536, 32, a.n
    X = synth(n, d, seed=0, dev=dev, kind=a.data)
    t0 = time.perf_counter()
    opq = OptimizedProductQuantizer(M=M, B=8)
    opq.niter = a.opq_iters
    opq.fit(X[:65536])
    torch.cuda.synchronize()
    t_fit = time.perf_counter() - t0
    C = opq.inner.centroids_device
    prep = _native.pq_prepare(C, 8)
    Y = torch.empty_like(X)
    codes = torch.empty((n, M), dtype=torch.uint8, device=dev)
    rot = lambda: opq.opq.rotate(X, False, out=Y)  # noqa: E731

    def step():
        rot()
        _native.pq_encode(Y, C, prep, 8, out=codes)

    wall, dev_ms = timed(step, steps, warmup)
    _, rot_ms = timed(rot, steps, 1)
    Q = X[:a.nq].contiguous()  # the reference's convention: queries are the first rows

    def search():
        lut = _native.adc_lut(opq.opq.rotate(Q, False), C, 8)
        return _native.adc_search(lut, codes, 10, 8)

    swall, _ = timed(search, 3, 1)
    _, ai = search()
    _, gi = _native.flat_search(Q[:100].contiguous(), X, 10)
    Xhat = opq.opq.rotate(_native.pq_decode(codes, C, 8), True)
    _, di = _native.flat_search(Q[:100].contiguous(), Xhat, 10)
    del Xhat
    cpu_b = opq32_cpu_baseline(X, Y, codes, opq.opq.A_device, C, a.cpu_seconds / 2) if cpu else None
    del X, Y
    g, r, dd = (t.cpu().numpy() for t in (gi, ai[:100], di))
    rec = lambda ref, x: float(np.mean([len(set(ref[j]) & set(x[j])) / 10 for j in range(len(ref))]))  # noqa: E731
    flops = 2.0 * d * d * n  # the fp32 GEMM's flops (algorithmic)
    tfs = flops / (rot_ms * 1e-3) / 1e12
    split = _native.opq_prepare(opq.opq.A_device) is not None
    # the split-f16 kernel spends 3 f16 MFMAs per fp32-accurate multiply-add: its ceiling is
    # the dense f16 peak / 3; the plain fp32 MFMA kernel's is the fp32 matrix peak
    peak = MFMA_F16_PEAK_TFS / 3 if split else MFMA_F32_PEAK_TFS
    return {"metric": "OPQ32 encode vectors/sec + ADC queries/sec @ recall@10, 1M×1536 fp32 (BASELINE configs[2])",
            "value": n / wall, "unit": "vectors/s", "ms_per_step": wall * 1e3, "dtype": "f32",
            "config": {"workload": f"opq32_encode_{n}x{d}", "M": M, "nbits": 8, "opq_outer_iters": a.opq_iters,
                       "fit_s": t_fit, "data": a.data},
            "roofline": {"bound": "mfma", "kernel": _native.opq_backend(d) if split else "opq_gemm_kernel (fp32 MFMA)",
                         "achieved": tfs, "peak": peak, "unit": "TFLOP/s (fp32-accurate)", "frac": tfs / peak,
                         "peak_note": "dense f16 MFMA peak / 3 (x_hi b_hi + x_hi b_lo + x_lo b_hi)" if split else
                                      "dense fp32 MFMA peak", "vs_fp32_mfma_peak": tfs / MFMA_F32_PEAK_TFS,
                         "rotate_ms": rot_ms, "encode_call_ms": dev_ms - rot_ms,
                         "traffic": traffic_from_profile(f"opq32_rotate_{n}x{d}")},
            "adc": {"qps": a.nq / swall, "nq": a.nq, "k": 10, "recall@10": rec(g, r), "recall_queries": 100,
                    "recall@10_decode_exact": rec(g, dd), "topk_agreement_adc_vs_decode_exact": rec(dd, r),
                    "ms_per_batch": swall * 1e3},
            **({"cpu_baseline": cpu_b} if cpu_b else {})}


def opq32_cpu_baseline(X, Y, codes, A, C, target_s):
    """OPQ encode on the host cores, as the reference's path runs it: the rotation x A^T as a BLAS
    sgemm (numpy; faiss OPQMatrix.apply, optimized_product_quantization.py:30-31) followed by the
    oracle's OpenMP PQ encode (faiss compute_codes), on a bounded sample of the same rows.
    Checks: the oracle's encode of the GPU-rotated sample equals the GPU codes bit for bit; the
    CPU-rotated sample's codes agree except at near-ties of the two roundings (fraction)."""
    O = _oracle()
    Ah, Cn = A.cpu().numpy(), C.cpu().numpy()
    fn = lambda xs: O.pq_encode(np.ascontiguousarray(xs @ Ah.T), Cn)  # noqa: E731
    n_cal = 1000
    t0 = time.perf_counter()
    fn(X[:n_cal].cpu().numpy())
    dt = time.perf_counter() - t0
    n_s = int(min(X.shape[0], max(n_cal, n_cal * target_s / max(dt, 1e-6))))
    Xs = X[:n_s].cpu().numpy()
    t0 = time.perf_counter()
    ref_cpu = fn(Xs)
    dt = time.perf_counter() - t0
    got = codes[:n_s].cpu().numpy()
    ref_gpu_rot = O.pq_encode(Y[:n_s].cpu().numpy(), Cn)
    return {"value": n_s / dt, "unit": "vectors/s", "cores": O.cpu_threads(), "kind": "port",
            "sample": f"first {n_s} rows: numpy sgemm rotation + oracle pq_encode (OpenMP), {dt:.1f} s wall",
            "codes_equal_gpu_on_gpu_rotation": bool(np.array_equal(got, ref_gpu_rot)),
            "code_agreement_cpu_rotation": float((got == ref_cpu).mean())}


def pq_wide_leg(a, dev, M, steps, warmup, cpu=True):
    """The sweep's own PQ shape (BASELINE configs[0]: `vq-benchmark sweep --method pq` on 1536-d
    dbpedia rows, M = 8 -> dsub 192): the wide-subspace filter (K in two tile halves) + resolve,
    1M x 1536 Gaussian rows, parity against the oracle on a 200,000-row sample."""
    d, n = 1536, a.n
    X = synth(n, d, seed=3, dev=dev, kind="gaussian")
    C = train_codebook(X, M, 8, 0, 1, dev)
    codes, e = encode_leg(X, C, a, 0, 1, dev, steps, warmup)
    pa = parity_check(X, C, codes, _oracle(), max_rows=200_000, fp64_rows=5000)[0] if cpu else None
    cb = cpu_baseline(X, C, _oracle(), a.cpu_seconds / 2) if cpu else None
    del X, codes
    return {"metric": f"PQ{M} encode vectors/sec, 1M×1536 fp32 (the sweep's PQ shape, BASELINE configs[0])",
            "value": n / e["wall_s"], "unit": "vectors/s", "ms_per_step": e["wall_s"] * 1e3, "dtype": "f32",
            "config": {"workload": f"pq{M}_encode_{n}x{d}", "M": M, "dsub": d // M, "nbits": 8, "data": "gaussian"},
            "roofline": {"bound": "hbm", "achieved": e["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": e["achieved_gbs"] / HBM_PEAK_GBS, "bytes_per_vector": e["bytes_per_vector"],
                         "kernel_ms": e["kernel_ms"], "traffic": traffic_from_profile(f"pq{M}_encode_{n}x{d}"),
                         "traffic_note": "PMC HBM bytes of the filter + resolve launches (the code transpose, ~1 %, not included)",
                         "kernel": "pq_encode_cs_kernel (K-halves filter, 8 waves) + pq_resolve_merged_kernel + transpose"},
            "parity": pa, **({"cpu_baseline": cb} if cb else {})}


def flatcodes_leg(a, dev, kind, steps, warmup, cpu=True):
    d, n = 3072, a.n
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    X = torch.randn((n, d), generator=g, device=dev, dtype=torch.float32)
    if kind == "sq8":
        lo, hi = X.amin(0), X.amax(0)
        den = (hi - lo) + 1e-8
        enc = lambda: _native.sq_encode(X, lo, den, 8)  # noqa: E731
        dec = lambda c: _native.sq_decode(c, d, lo, den, 8)  # noqa: E731
        bpv, kname = 4 * d + d, "sq_encode_f32_vec_kernel"
    else:
        enc = lambda: _native.rabitq_encode(X, None, _native.METRIC_L2)  # noqa: E731
        dec = lambda c: _native.rabitq_decode(c, d, None)  # noqa: E731
        bpv, kname = 4 * d + d // 8 + 8, "rabitq_encode_wide_kernel<6>"
    wall, dev_ms = timed(enc, steps, warmup)
    codes = enc()
    # this box's streaming rates on the same bytes (torch device copy: read + write; sum: read):
    # the spec peak is the roofline, these say how much of it a plain stream gets here
    Y = torch.empty_like(X)
    _, copy_ms = timed(lambda: Y.copy_(X), 5, 2)
    del Y
    _, read_ms = timed(lambda: X.sum(), 5, 2)
    calib = {"copy_gbs": 2 * X.numel() * 4 / (copy_ms * 1e-3) / 1e9, "read_gbs": X.numel() * 4 / (read_ms * 1e-3) / 1e9,
             "note": "torch Y.copy_(X) (read + write) and X.sum() (read) on the leg's input, same box"}
    Q = X[:100].contiguous()  # reference convention: the queries are the first database rows
    search = lambda: _native.flat_search(Q, dec(codes), 10)  # noqa: E731
    swall, _ = timed(search, 2, 1)
    _, ai = search()
    _, gi = _native.flat_search(Q, X, 10)
    rec = lambda ref, x: float(np.mean([len(set(ref[j]) & set(x[j])) / 10 for j in range(len(ref))]))  # noqa: E731
    g_, r_ = gi.cpu().numpy(), ai.cpu().numpy()
    ach = n * bpv / (dev_ms * 1e-3) / 1e9
    out = {"metric": f"{kind} encode vectors/sec + search queries/sec @ recall@10, 1M×3072 fp32 (BASELINE configs[3])",
           "value": n / wall, "unit": "vectors/s", "ms_per_step": wall * 1e3, "dtype": "f32",
           "config": {"workload": f"{kind}_encode_{n}x{d}"},
           "roofline": {"bound": "hbm", "kernel": kname, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS, "bytes_per_vector": bpv, "kernel_ms": dev_ms,
                        "traffic": traffic_from_profile(f"{kind}_encode_{n}x{d}"),
                        "box_stream_rates": calib, "frac_of_box_copy_rate": ach / calib["copy_gbs"]},
           "search": {"qps": 100 / swall, "nq": 100, "k": 10, "recall@10": rec(g_, r_),
                      "method": "decode + exact L2 scan of the reconstructions (the reference's flat search)"}}
    if kind == "rabitq1":  # RaBitQIndex: IndexRaBitQ estimator search (center = mean, qb = 4)
        center = X.double().mean(0).float().contiguous()
        codes_c = _native.rabitq_encode(X, center, _native.METRIC_L2)
        Qe = X[: a.nq].contiguous()
        est = lambda: _native.rabitq_search(codes_c, d, center, Qe, 4, _native.METRIC_L2, 10)  # noqa: E731
        ewall, _ = timed(est, 3, 1)
        _, ei = est()
        # the integer dots <bits, q'> of every (query, code) pair on v_mfma_i32_32x32x32_i8: 2 d ops
        # per pair over the whole search (query prep, first-block top-k and merges included)
        tops = 2.0 * a.nq * n * d / ewall / 1e12
        out["estimator_search"] = {"qps": a.nq / ewall, "nq": a.nq, "k": 10, "qb": 4, "ms_per_batch": ewall * 1e3,
                                   "recall@10": rec(g_, ei[:100].cpu().numpy()),
                                   "roofline": {"bound": "mfma", "achieved": tops, "peak": INT8_MFMA_PEAK_TOPS,
                                                "unit": "TOPS", "frac": tops / INT8_MFMA_PEAK_TOPS,
                                                "ops_per_pair": 2 * d},
                                   "method": "mivq_rabitq_search: int8 MFMA over sign bits (128 queries per "
                                             "workgroup) + estimator; dense first block + tiled top-k, then "
                                             "screened blocks (keys kept only below the running k-th) merged in place"}
    if cpu:
        out["cpu_baseline"] = flatcodes_cpu_baseline(kind, X, codes, lo if kind == "sq8" else None,
                                                     den if kind == "sq8" else None, a.cpu_seconds / 2)
    del X
    return out


def flatcodes_cpu_baseline(kind, X, codes, lo, den, target_s):
    """The reference's CPU path for these encoders on a bounded sample of the same rows: SQ-8 as
    ScalarQuantizer._compress_block writes it in numpy (scalar_quantization.py:52-68, one
    thread), RaBitQ-1 as the oracle's OpenMP restatement of faiss RaBitQuantizer.compute_codes
    (rabit_quantization.py:25-26); the sample's GPU codes must equal the CPU's."""
    O = _oracle()
    if kind == "sq8":
        lo_h, den_h = lo.cpu().numpy(), den.cpu().numpy()
        fn = lambda xs: O.sq_encode_numpy(xs, lo_h, den_h, 8)  # noqa: E731
        cores, how = 1, "numpy restatement of ScalarQuantizer._compress_block (oracle.sq_encode_numpy)"
    else:
        fn = lambda xs: O.rabitq_encode(xs)  # noqa: E731
        cores, how = O.cpu_threads(), "oracle/mivq_oracle.c rabitq_encode (OpenMP)"
    n_cal = 2000
    t0 = time.perf_counter()
    fn(X[:n_cal].cpu().numpy())
    dt = time.perf_counter() - t0
    n_s = int(min(X.shape[0], max(n_cal, n_cal * target_s / max(dt, 1e-6))))
    Xs = X[:n_s].cpu().numpy()
    t0 = time.perf_counter()
    ref = fn(Xs)
    dt = time.perf_counter() - t0
    got = codes[:n_s].cpu().numpy()
    if kind == "sq8":
        equal = bool(np.array_equal(got, ref))
    else:  # sign bits exact, the two f32 factors within 1e-5 relative (faiss-internal order)
        nb = (X.shape[1] + 7) // 8
        f_g, f_r = got[:, nb:].copy().view(np.float32), ref[:, nb:].copy().view(np.float32)
        equal = bool(np.array_equal(got[:, :nb], ref[:, :nb]) and
                     np.all(np.abs(f_g - f_r) <= 1e-5 * np.maximum(np.abs(f_r), 1e-30)))
    return {"value": n_s / dt, "unit": "vectors/s", "cores": cores, "kind": "port",
            "sample": f"first {n_s} rows, {how}, {dt:.1f} s wall", "codes_equal_gpu": equal}


def extrabitq_leg(a, dev, steps, warmup, cpu=True):
    """The registry's `rabitq` route (method_registry_saq.py:45-48 -> ExtendedRaBitQuantizer,
    extended_rabitq.py:125-199): B-bit encode + decode of synthetic Gaussian rows at D = 3072.
    A step is one round trip (compress + decompress); the roofline is erq_rotate_kernel's fp64
    MFMA GEMM (2 D^2 FLOP per vector per direction), timed alone with HIP events on the stream
    it runs on.  CPU baseline: the reference's numpy algorithm (oracle.extrabitq_encode, fp64
    BLAS matmul) on a bounded sample, BLAS threads pinned with threadpoolctl."""
    from haag_vq.methods.extended_rabitq import ExtendedRaBitQuantizer

    d, n, nbits = 3072, a.erq_rows, 4
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    X = torch.randn((n, d), generator=g, device=dev, dtype=torch.float32)
    t0 = time.perf_counter()
    q = ExtendedRaBitQuantizer(num_bits=nbits, seed=0)
    q.fit(X)
    c, P, lv = q._state()
    t_fit = time.perf_counter() - t0
    codes = q.compress(X)
    wall, dev_ms = timed(lambda: q.decompress(q.compress(X)), steps, warmup)
    _, enc_ms = timed(lambda: q.compress(X), steps, 1)
    o = torch.randn((n, d), generator=g, device=dev, dtype=torch.float64)
    _, rot_ms = timed(lambda: _native.extrabitq_rotate(o, P, False), steps, 1)
    _, rotT_ms = timed(lambda: _native.extrabitq_rotate(o, P, True), steps, 1)
    del o
    flops = 2.0 * n * d * d
    tfs = flops / (rot_ms * 1e-3) / 1e12
    xh = q.decompress(codes)
    rel = float(((xh.double() - X.double()).norm(dim=1) / X.double().norm(dim=1)).mean())
    out = {"metric": "Extended RaBitQ (registry `rabitq`) encode+decode vectors/sec, 3072-d fp32",
           "value": n / wall, "unit": "vectors/s", "ms_per_step": wall * 1e3, "dtype": "f64",
           "config": {"workload": f"extrabitq{nbits}_roundtrip_{n}x{d}", "num_bits": nbits, "fit_s": t_fit,
                      "encode_ms": enc_ms, "step": "compress + decompress"},
           "roofline": {"bound": "mfma", "kernel": "erq_rotate_fast_kernel (v_mfma_f64_16x16x4_f64, o . P)",
                        "achieved": tfs, "peak": MFMA_F64_PEAK_TFS, "unit": "TFLOP/s", "frac": tfs / MFMA_F64_PEAK_TFS,
                        "rotate_ms": rot_ms, "rotate_transposed_ms": rotT_ms, "flops_per_launch": flops,
                        "flops_per_vector": 2 * d * d,
                        "peak_note": "MI355X dense fp64 matrix spec (78.6 TF); not in the microarch guide's table"},
           "reconstruction_rel_err_mean": rel}
    if cpu:
        out["cpu_baseline"] = extrabitq_cpu_baseline(X, codes, q, a.cpu_seconds / 2)
    del X, codes, xh
    return out


def extrabitq_cpu_baseline(X, codes, q, target_s):
    """extended_rabitq.py:125-170 in numpy on the host cores (oracle.extrabitq_encode: fp64 BLAS
    rotation), on a bounded sample of the same rows.  The sample's GPU indices must equal the CPU's
    except where s sits on a level midpoint (fp64 summation order: tests/test_pinning_gpu.py)."""
    from threadpoolctl import threadpool_limits

    O = _oracle()
    threads = O.cpu_threads()
    nb = q.num_bits
    fn = lambda xs: O.extrabitq_encode(xs, q.c, q.P, q.levels, nb)  # noqa: E731
    with threadpool_limits(limits=threads):
        n_cal = 500
        t0 = time.perf_counter()
        fn(X[:n_cal].cpu().numpy())
        dt = time.perf_counter() - t0
        n_s = int(min(X.shape[0], max(n_cal, n_cal * target_s / max(dt, 1e-6))))
        Xs = X[:n_s].cpu().numpy()
        t0 = time.perf_counter()
        ref = fn(Xs)
        dt = time.perf_counter() - t0
    got = codes[:n_s].cpu().numpy()
    D = Xs.shape[1]
    ib = (D * nb + 7) // 8

    def unpack(cb):
        bits = np.unpackbits(cb[:, :ib], axis=1)[:, :D * nb].reshape(len(cb), D, nb)
        return (bits.astype(np.int64) << np.arange(nb - 1, -1, -1)).sum(-1)

    gi, ri = unpack(got), unpack(ref)
    bad = np.argwhere(gi != ri)
    ties = 0
    if len(bad):
        Xb = Xs[np.unique(bad[:, 0])].astype(np.float64)
        rows = {r: i for i, r in enumerate(np.unique(bad[:, 0]))}
        r_ = Xb - q.c
        o_ = r_ / np.maximum(np.linalg.norm(r_, axis=1), 1e-12)[:, None]
        s_ = (o_ @ q.P) * np.sqrt(D)
        mids = 0.5 * (q.levels[:-1] + q.levels[1:])
        for i, j in bad:
            v = s_[rows[i], j]
            ties += int(np.min(np.abs(mids - v)) <= 1e-12 * max(1.0, abs(v)) and abs(int(gi[i, j]) - int(ri[i, j])) == 1)
    f_g, f_r = got[:, ib:].copy().view(np.float32), ref[:, ib:].copy().view(np.float32)
    return {"value": n_s / dt, "unit": "vectors/s (encode)", "cores": threads, "kind": "port",
            "sample": f"first {n_s} rows, oracle.extrabitq_encode (numpy fp64, BLAS on {threads} threads via "
                      f"threadpoolctl), {dt:.1f} s wall",
            "index_mismatches": int(len(bad)), "index_mismatches_that_are_midpoint_ties": ties,
            "indices_compared": int(gi.size),
            "factors_max_rel_diff": float(np.max(np.abs(f_g - f_r) / np.maximum(np.abs(f_r), 1e-30)))}


def config5_leg(a, rank, world, dev, steps, warmup):
    """BASELINE configs[4]: 53.2M x 1024 row-sharded (6.65M rows per GPU), PQ16 + ADC top-10."""
    n, d, M = a.config5_rows, 1024, 16
    X = synth(n, d, seed=100 + rank, dev=dev, kind=a.data)
    C = train_codebook(X, M, 8, rank, world, dev)
    codes, enc = encode_leg(X, C, a, rank, world, dev, steps, warmup)
    Q = X[:a.config5_nq].clone() if rank == 0 else torch.empty((a.config5_nq, d), dtype=torch.float32, device=dev)
    adc = adc_leg(X, C, codes, a, rank, world, dev, Q, a.k, a.gt_queries, reps=2, cpu=False)
    frac = enc["achieved_gbs"] / HBM_PEAK_GBS
    del X, codes
    return {"metric": "PQ16 encode vectors/sec + ADC queries/sec @ recall@10, 53.2M×1024 row-sharded (BASELINE configs[4])",
            "value": world * n / enc["wall_s"], "unit": "vectors/s", "n_gpus": world, "rows_per_gpu": n,
            "rows_total": world * n, "ms_per_step": enc["wall_s"] * 1e3, "scaling": "weak",
            "roofline": {"bound": "hbm", "achieved": enc["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": frac, "bytes_per_vector": enc["bytes_per_vector"], "kernel_ms": enc["kernel_ms"]},
            "adc": adc}


# ------------------------------------------------------------------------- dry run (CPU)
def dry_run(a):
    """The launcher and rank plumbing over gloo on CPU tensors: codebook and query broadcast,
    per-shard exact top-k with global ids, all-gather + (dist, id) merge; rank 0 checks the
    merged lists against the single-rank answer.  No GPU and no timing: a harness check."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    n_per, d, M, k, nq = 300, 32, 4, a.k, 5
    shards = [np.random.default_rng(r).standard_normal((n_per, d)).astype(np.float32) for r in range(world)]
    C = torch.from_numpy(np.random.default_rng(99).standard_normal((M, 256, d // M)).astype(np.float32))
    C = sharded.broadcast_(C if rank == 0 else torch.zeros_like(C))
    Q = torch.from_numpy(np.random.default_rng(7).standard_normal((nq, d)).astype(np.float32))
    Q = sharded.broadcast_(Q if rank == 0 else torch.zeros_like(Q))

    def topk(Xs, off):
        dd = ((Q.double()[:, None, :] - torch.from_numpy(Xs).double()[None]) ** 2).sum(-1)
        ids = torch.arange(off, off + Xs.shape[0], dtype=torch.int64).expand_as(dd)
        o = np.lexsort((ids.numpy(), dd.numpy()))[:, :k]
        return (torch.from_numpy(np.take_along_axis(dd.numpy(), o, 1).astype(np.float32)),
                torch.from_numpy((o + off).astype(np.uint32).view(np.int32)))

    def merge(gd, gi, kk):
        P, q_, _ = gd.shape
        dd = gd.permute(1, 0, 2).reshape(q_, -1).numpy()
        ii = gi.permute(1, 0, 2).reshape(q_, -1).numpy().view(np.uint32).astype(np.int64)
        o = np.lexsort((ii, dd))[:, :kk]
        return (torch.from_numpy(np.take_along_axis(dd, o, 1)),
                torch.from_numpy(np.take_along_axis(ii, o, 1).astype(np.uint32).view(np.int32)))

    ld, li = topk(shards[rank], rank * n_per)
    gd, gi = sharded.exchange_topk(ld, li, k, merge=merge)
    if rank == 0:
        sd, si = topk(np.concatenate(shards), 0)
        same = bool(torch.equal(gi, si) and torch.equal(gd, sd))
        print(json.dumps({"metric": METRIC, "value": None, "unit": "vectors/s", "n_gpus": world, "dry_run": True,
                          "merged_equals_single": same, "codebook_checksum": float(C.double().sum()),
                          "config": {"workload": "dry-run", "rows_per_rank": n_per, "parallelism": f"row-sharded x{world}"}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


# ------------------------------------------------------------------------- main
def summary_of(out, k):
    """Compact digest of the bench line: the encode headline and the ADC headline (queries/s,
    recall@k, roofline frac), and the same few figures of the north-star, config #5 and
    configs legs."""
    def r(x, n=4):
        return None if x is None else round(float(x), n)

    def adc_digest(ad):
        if not ad:
            return None
        rf = ad.get("roofline") or {}
        return {"qps": r(ad["qps"], 0), f"recall@{k}": r(ad.get(f"recall@{k}")), "frac": r(rf.get("frac")),
                "bound": rf.get("bound"), "scan_ms": r(rf.get("scan_ms"))}

    sm = {"encode_vps": r(out["value"], 0), "encode_frac": r(out["roofline"]["frac"]),
          "parity_mismatched_codes": (out.get("parity_sample") or {}).get("mismatched_codes"),
          "adc": adc_digest(out.get("adc"))}
    ns = out.get("north_star")
    if ns:
        sm["north_star"] = {"vps": r(ns["value"], 0), "frac": r(ns["roofline"]["frac"])}
    c5 = out.get("config5")
    if c5:
        sm["config5"] = {"vps_per_gpu": r(c5.get("value_per_gpu", c5.get("value")), 0),
                         "frac": r((c5.get("roofline") or {}).get("frac")), "adc": adc_digest(c5.get("adc"))}
    cf = out.get("configs") or {}
    for name, leg in cf.items():
        if isinstance(leg, dict):
            sm[name] = {"value": r(leg.get("value"), 0), "frac": r((leg.get("roofline") or {}).get("frac"))}
            es = leg.get("estimator_search")
            if es:
                sm[name]["estimator_qps"] = r(es["qps"], 0)
                sm[name]["estimator_frac"] = r((es.get("roofline") or {}).get("frac"))
    return sm


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if a.gpus > 1 and env_world is None:
        return launch_ranks(a)  # before anything touches the GPU
    world = int(env_world or "1")
    if env_world is not None and a.gpus not in (1, world):
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    if a.dry_run:
        dry_run(a)
        return 0
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one process per GPU; VQ_DIST_BACKEND=gloo rehearses the same ranks sharing a GPU
        # (host-staged collectives, tests/test_sharded_gpu.py) -- RCCL otherwise
        gpu = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(gpu)
        if os.environ.get("VQ_DIST_BACKEND", "nccl") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dev = _native.require_device()
    head_only = rank == 0 and world == 1

    log(f"[rank {rank}] generating {a.n}x{a.d} ({a.data}) on {torch.cuda.get_device_name(dev)}")
    X = synth(a.n, a.d, seed=rank, dev=dev, kind=a.data)
    C = train_codebook(X, a.M, 8, rank, world, dev)
    codes, enc = encode_leg(X, C, a, rank, world, dev, a.steps, a.warmup, exact=a.exact, legacy=a.legacy)
    value = world * a.n / enc["wall_s"]
    log(f"[rank {rank}] encode: {enc['wall_s'] * 1e3:.3f} ms/step wall, {enc['kernel_ms']:.3f} ms/call device")
    workload = f"pq{a.M}_encode_{a.n}x{a.d}"

    parity = cpu = None
    if head_only and not a.no_cpu_baseline:
        O = _oracle()
        parity, _ = parity_check(X, C, codes, O)
        cpu = cpu_baseline(X, C, O, a.cpu_seconds)
        log(f"[rank 0] parity {parity}; cpu baseline {cpu}")

    adc = None
    if not a.no_adc:
        # queries = the first database rows of rank 0's shard, the reference's convention
        # (data/datasets.py:79-81, dbpedia_loader.py:222); broadcast to every rank
        Q = X[:a.nq].clone() if rank == 0 else torch.empty((a.nq, a.d), dtype=torch.float32, device=dev)
        adc = adc_leg(X, C, codes, a, rank, world, dev, Q, a.k, a.gt_queries, cpu=not a.no_cpu_baseline)
        if rank == 0:
            log(f"[rank 0] adc: {adc}")
    del X, codes

    alt = None
    if head_only and not a.no_alt_data:
        kind = "clustered" if a.data == "gaussian" else "gaussian"
        Xa = synth(a.n, a.d, seed=7, dev=dev, kind=kind)
        Ca = train_codebook(Xa, a.M, 8, 0, 1, dev)
        ca, ea = encode_leg(Xa, Ca, a, 0, 1, dev, a.steps, a.warmup)
        pa = parity_check(Xa, Ca, ca, _oracle(), max_rows=200_000, fp64_rows=5000)[0] if not a.no_cpu_baseline else None
        alt = {"data": kind, "value": a.n / ea["wall_s"], "unit": "vectors/s", "ms_per_step": ea["wall_s"] * 1e3,
               "kernel_ms": ea["kernel_ms"], "roofline_frac": ea["achieved_gbs"] / HBM_PEAK_GBS, "parity": pa}
        if not a.no_adc:
            # the ADC leg on these rows too: recall@k means more on clustered rows than on
            # isotropic ones, and the filter certifies a different share of the queries
            aa = adc_leg(Xa, Ca, ca, a, 0, 1, dev, Xa[:a.nq].clone(), a.k, a.gt_queries, cpu=False)
            alt["adc"] = {key: aa[key] for key in ("qps", "nq", "k", f"recall@{a.k}", f"recall@{a.k}_decode_exact",
                                                   "topk_agreement_adc_vs_decode_exact", "ms_per_batch")}
            alt["adc"]["scan_ms"] = aa["roofline"]["scan_ms"]
            alt["adc"]["roofline_frac"] = aa["roofline"]["frac"]
        log(f"[rank 0] alt data: {alt}")
        del Xa, ca

    ns = None
    if head_only and not a.no_north_star and a.north_star_rows > a.n:
        Xn = synth(a.north_star_rows, a.d, seed=11, dev=dev, kind="gaussian")
        Cn = train_codebook(Xn, a.M, 8, 0, 1, dev)
        cn_, en = encode_leg(Xn, Cn, a, 0, 1, dev, 5, 1)
        pn = None
        if not a.no_cpu_baseline:
            pn = parity_check(Xn, Cn, cn_, _oracle(), max_rows=200_000, fp64_rows=5000)[0]
        ns = {"workload": f"pq{a.M}_encode_{a.north_star_rows}x{a.d}", "data": "gaussian",
              "value": a.north_star_rows / en["wall_s"], "unit": "vectors/s", "ms_per_step": en["wall_s"] * 1e3,
              "steps": 5, "warmup": 1, "kernel_ms": en["kernel_ms"],
              "roofline": {"bound": "hbm", "achieved": en["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": en["achieved_gbs"] / HBM_PEAK_GBS, "bytes_per_vector": en["bytes_per_vector"]},
              "parity": pn}
        log(f"[rank 0] north star: {ns}")
        del Xn, cn_
        torch.cuda.empty_cache()

    c5 = None
    if not a.no_config5:
        c5 = config5_leg(a, rank, world, dev, a.steps, a.warmup)
        if rank == 0:
            log(f"[rank 0] config5: {c5}")

    configs = None
    if head_only and not a.no_configs:
        configs = {}
        cb = not a.no_cpu_baseline
        for name, fn in (("pq8", lambda: pq_wide_leg(a, dev, 8, 10, 3, cpu=cb)),
                         ("opq32", lambda: opq32_leg(a, dev, 3, 1, cpu=cb)),
                         ("sq8", lambda: flatcodes_leg(a, dev, "sq8", 5, 2, cpu=cb)),
                         ("rabitq1", lambda: flatcodes_leg(a, dev, "rabitq1", 5, 2, cpu=cb)),
                         ("extrabitq4", lambda: extrabitq_leg(a, dev, 3, 1, cpu=cb))):
            configs[name] = fn()
            torch.cuda.empty_cache()
            log(f"[rank 0] {name}: {configs[name]}")

    if rank == 0:
        frac = enc["achieved_gbs"] / HBM_PEAK_GBS
        tkey = f"{workload}_{a.data}"
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "vectors/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": enc["wall_s"] * 1e3,
            "warmup_settle": {"ms": SETTLE_MS, "extra_untimed_steps": SETTLE["extra_steps"],
                              "why": "after the W warmup calls, untimed calls continue until the GPU has been busy "
                                     "for this long (power-management transient, see timed())"},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic {a.data} (see synth(): generated on device, seed = rank, rows L2-normalised); "
                    "codebooks from GPU k-means on the first 65,536 rows (seed 1234, 25 iterations)",
            "config": {"workload": workload, "rows_per_gpu": a.n, "dim": a.d, "M": a.M, "nbits": 8,
                       "path": "exact" if a.exact else ("legacy-mfma" if a.legacy else "cs-mfma-filter+exact-recheck"),
                       "data": a.data, "parallelism": f"row-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": enc["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": frac, "traffic": traffic_from_profile(tkey),
                         "kernel": "mivq_pq_encode call: pq_encode_cs_kernel (fp16-MFMA filter + pair window) + "
                                   "pq_resolve_merged_kernel (canonical fp32 re-check of the row-subspaces the filter "
                                   "could not settle) + pq_transpose_codes16_kernel",
                         "bytes_per_vector": enc["bytes_per_vector"], "kernel_ms": enc["kernel_ms"]},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "adc": adc,
            "alt_data": alt,
            "north_star": ns,
            "config5": c5,
            "configs": configs,
        }
        # LAST key (a driver keeps the tail of this one long line): the headline numbers of
        # every leg in a few hundred bytes
        out["summary"] = summary_of(out, a.k)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
