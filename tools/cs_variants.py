"""Time the codebook-stationary encode kernel with parts of its work removed.

usage: python tools/cs_variants.py [--n 1000000] [--reps 10]
Builds tools/build/libcsvar.so (hipcc, gfx950) unless it exists, then prints one line per
variant: device ms per launch (HIP events on the launch stream).
"""
import argparse
import ctypes
import subprocess
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from bench import synth  # noqa: E402

VARIANTS = {0: "encode + resolve", 1: "encode only", 2: "resolve: pairs only", 4: "resolve: full scans only",
            8: "resolve: gathers, no compute", 33: "encode only, 1 of 8 cb",
            17: "loads + convert + tile + fragments only", 65: "encode only, no x loads (compute alone)",
            145: "streaming only, subspace-major probe", 256: "encode + resolve, 256-wide full scans",
            513: "encode + full-item kernel", 1537: "... no exact chains", 2561: "... 1 of 8 filter blocks",
            4609: "... no gathers", 7681: "... none of the three", 16384: "encode + resolve, lane-wide top-3 filter", 32768: "encode + resolve, no pair window", 65536: "encode + resolve, LDS-codebook full-item kernel",
            131073: "encode only, A fragments of block 0 reused (LDS probe)", 131072: "encode + resolve, A fragments reused",
            1048576: "round-1 resolve (pair window in the pair kernel, full2 + pair kernels)"}


def prep_layout(M, dsub, ksub=256):
    """Byte offsets inside the mivq_pq_prepare buffer (mirror of PqPrepLayout, mivq_common.h)."""
    al = lambda v: (v + 255) // 256 * 256  # noqa: E731
    ks = (dsub + 15) // 16
    L, off = {}, 0
    L["cn"] = off; off = al(off + 4 * M * ksub)
    L["ct"] = off; off = al(off + 4 * M * dsub * ksub)
    L["img"] = off; off = al(off + M * 8 * ks * 64 * 8 * 2)
    L["hinit"] = off; off = al(off + 4 * M * ksub)
    L["bnd"] = off; off = al(off + 4 * M * 4)
    L["spread"] = off; off = al(off + 4 * M * 2)
    L["pd"] = off; off = al(off + (M * 256 * 256 * 8 if M <= 64 else 0))
    L["bnd2"] = off
    return L


def build(lib=None):
    """tools/build/libcsvar.so (all variants), or --lib: a prebuilt one, e.g. built with only the
    variants at hand:  hipcc ... -DCS_VARIANTS="VARIANT(0) VARIANT(1)" -o tools/build/x.so"""
    if lib:
        return ctypes.CDLL(str(ROOT / lib))
    so = ROOT / "tools" / "build" / "libcsvar.so"
    src = ROOT / "tools" / "cs_variants.hip"
    if not so.exists() or so.stat().st_mtime < max(src.stat().st_mtime, (ROOT / "vector-quantization_amd/csrc/pq_encode_cs.hip").stat().st_mtime):
        so.parent.mkdir(exist_ok=True)
        subprocess.check_call(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                               "-ffp-contract=off", "-fvisibility=hidden", "-o", str(so), str(src)])
    return ctypes.CDLL(str(so))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--data", default="clustered")
    ap.add_argument("--ab", default="", help="V1,V2: interleaved A/B timing instead of the variant table")
    ap.add_argument("--lib", default="", help="prebuilt harness library (e.g. another MIVQ_CS_WAVES)")
    ap.add_argument("--ab-lib", default="", help="other harness library: interleaved A/B of V=--ab-v in both")
    ap.add_argument("--ab-v", type=int, default=0)
    a = ap.parse_args()
    lib = build(a.lib)
    dev = _native.require_device()
    X = synth(a.n, a.d, 0, dev, kind=a.data)
    probes(lib, X, a.reps)
    C = train_pq(X[:65536], a.M, 8, niter=25, seed=1234).contiguous()
    prep = _native.pq_prepare(C, 8)
    ref = _native.pq_encode(X, C, prep, 8)
    dsub = a.d // a.M
    L = prep_layout(a.M, dsub)
    base = prep.data_ptr()
    codesT = torch.empty((a.M, a.n), dtype=torch.uint8, device=dev)
    items = torch.empty((a.M * a.n * 8,), dtype=torch.uint8, device=dev)
    counts = torch.empty((a.M * a.n // 32 + 64, 2), dtype=torch.int32, device=dev)
    pinfo = torch.empty((a.M * a.n * 8,), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p

    def run(v, lib=lib):
        rc = lib.cs_variant(ctypes.c_int(v), P(X.data_ptr()), ctypes.c_int64(a.n), ctypes.c_int(a.d), ctypes.c_int(a.M),
                            ctypes.c_int(dsub), P(C.data_ptr()), P(base + L["cn"]), P(base + L["img"]),
                            P(base + L["hinit"]), P(base + L["bnd"]), P(base + L["pd"]), P(base + L["bnd2"]),
                            P(codesT.data_ptr()), P(items.data_ptr()), P(counts.data_ptr()), P(pinfo.data_ptr()),
                            P(st))
        assert rc == 0, rc

    if a.ab_lib:
        libs = {"this": lib, a.ab_lib: ctypes.CDLL(str(ROOT / a.ab_lib))}
        res = {k: [] for k in libs}
        for k, lb in libs.items():
            run(a.ab_v, lb)
        torch.cuda.synchronize()
        for _ in range(a.reps * 3):
            for k, lb in libs.items():
                s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s_.record(); run(a.ab_v, lb); e_.record()
                torch.cuda.synchronize()
                res[k].append(s_.elapsed_time(e_))
        for k in libs:
            t = sorted(res[k])
            print(f"AB lib={k} V={a.ab_v}: median {t[len(t) // 2]:.3f} ms  min {t[0]:.3f}  max {t[-1]:.3f}", flush=True)
        # back-to-back (no idle gap: the power-managed clock of a sustained run)
        for k, lb in libs.items():
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                run(a.ab_v, lb)
            s_.record()
            for _ in range(20):
                run(a.ab_v, lb)
            e_.record()
            torch.cuda.synchronize()
            print(f"AB lib={k} V={a.ab_v}: back-to-back {s_.elapsed_time(e_) / 20:.3f} ms/call", flush=True)
        return
    if a.ab:
        va, vb = (int(t) for t in a.ab.split(","))
        res = {va: [], vb: []}
        for v in (va, vb):
            run(v)
        torch.cuda.synchronize()
        for _ in range(a.reps * 3):
            for v in (va, vb):
                s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s_.record(); run(v); e_.record()
                torch.cuda.synchronize()
                res[v].append(s_.elapsed_time(e_))
        for v in (va, vb):
            t = sorted(res[v])
            print(f"AB V={v}: median {t[len(t) // 2]:.3f} ms  min {t[0]:.3f}  max {t[-1]:.3f}", flush=True)
        return
    # instrumentation: V=513 runs encode + the full-item kernel with counting (no pair
    # kernel); counts then hold the tallies
    counts.zero_()
    run(0)
    torch.cuda.synchronize()
    c0 = counts.clone()
    run(513)
    torch.cuda.synchronize()
    diff = (counts - c0).long()
    rows = int((diff[:, 0] & 0xFFFF).sum()); scans = int((diff[:, 0] >> 16).sum()); cands = int((diff[:, 1] >> 8).sum())
    print(f"full kernel: rows {rows}, whole-row scans {scans}, candidates {cands} ({cands / max(rows, 1):.2f}/row)",
          flush=True)
    run(262144)
    torch.cuda.synchronize()
    st_, ga_ = (int(v) for v in counts.long().sum(0).tolist())
    print(f"pair kernel: {st_} pairs settled by the pair window, {ga_} gathered "
          f"({st_ / max(st_ + ga_, 1):.1%} settled)", flush=True)
    for v, name in VARIANTS.items():
        run(v)
        torch.cuda.synchronize()
        if v == 0:
            ok = bool((codesT.t() == ref).all())
            counts.zero_()
            run(v)
            torch.cuda.synchronize()
            c = counts.sum(0).tolist()
            nz = counts[(counts.sum(1) > 0)].float()
            print(f"per-workgroup items: {nz.shape[0]} groups, pairs mean {nz[:, 0].mean():.0f} max {nz[:, 0].max():.0f}, "
                  f"full mean {nz[:, 1].mean():.0f} max {nz[:, 1].max():.0f}", flush=True)
            print(f"resolve items: pairs {c[0]} ({c[0] / (a.n * a.M):.2%} of row-subspaces), "
                  f"full {c[1]} ({c[1] / (a.n * a.M):.2%})", flush=True)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for s, e in ev:
            s.record(); run(v); e.record()
        torch.cuda.synchronize()
        ms = sorted(s.elapsed_time(e) for s, e in ev)[a.reps // 2]
        gbs = a.n * (4 * a.d + a.M) / (ms * 1e-3) / 1e9
        print(f"V={v:2d} {name:32s} {ms:7.3f} ms  {gbs:7.0f} GB/s" + (f"  codes match library: {ok}" if v == 0 else ""),
              flush=True)


def probes(lib, X, reps):
    out = torch.zeros(4, dtype=torch.int32, device=X.device)
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p
    names = {0: "1024x1024 thr, 4 loads/thr", 1: "512x1024, 8 loads/thr", 2: "256x768, 12 loads/thr",
             3: "4096x1024, 2 loads/thr"}
    for p, name in names.items():
        run = lambda: lib.read_probe(ctypes.c_int(p), P(X.data_ptr()), ctypes.c_int64(X.numel()), P(out.data_ptr()), P(st))  # noqa: E731
        run()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for s, e in ev:
            s.record(); run(); e.record()
        torch.cuda.synchronize()
        ms = sorted(s.elapsed_time(e) for s, e in ev)[reps // 2]
        print(f"read probe {name:28s} {ms:7.3f} ms  {X.numel() * 4 / (ms * 1e-3) / 1e9:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
