"""Time the merged resolve with parts of its work removed (the V bits of pq_resolve_merged_kernel),
for one subspace shape: filter alone (V=1), whole call (V=0), and the resolve without its full
batches, pair batches, chains, etc.  Builds tools/build/libcsvar_ks<KS>.so (CS_KS) if missing.

usage: python tools/resolve_split.py [--M 8] [--d 1536] [--n 1000000] [--reps 10]
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
from tools.cs_variants import prep_layout  # noqa: E402

VARIANTS = {1: "filter only", 0: "filter + merged resolve", 1 << 21: "resolve: no full batches",
            1 << 22: "resolve: no pair batches", (1 << 22) | (1 << 21): "resolve: setup only",
            1 << 23: "resolve: gathers only (no MFMA, no chains)", 1 << 24: "resolve: full batches without chains",
            1 << 25: "resolve: full batches, MFMA + window only"}


def build(ks):
    so = ROOT / "tools" / "build" / f"libcsvar_ks{ks}.so"
    if not so.exists():
        so.parent.mkdir(exist_ok=True)
        vs = " ".join(f"VARIANT({v})" for v in VARIANTS)
        subprocess.check_call(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                               "-ffp-contract=off", "-fvisibility=hidden", f"-DCS_KS={ks}", f"-DCS_VARIANTS={vs}",
                               "-o", str(so), str(ROOT / "tools" / "cs_variants.hip")])
    return ctypes.CDLL(str(so))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--build-only", action="store_true")
    a = ap.parse_args()
    dsub = a.d // a.M
    lib = build((dsub + 15) // 16)
    if a.build_only:
        return
    dev = _native.require_device()
    X = synth(a.n, a.d, 0, dev, kind="gaussian")
    C = train_pq(X[:65536], a.M, 8, niter=25, seed=1234).contiguous()
    prep = _native.pq_prepare(C, 8)
    ref = _native.pq_encode(X, C, prep, 8)
    L = prep_layout(a.M, dsub)
    base = prep.data_ptr()
    codesT = torch.empty((a.M, a.n), dtype=torch.uint8, device=dev)
    items = torch.empty((a.M * a.n * 8,), dtype=torch.uint8, device=dev)
    counts = torch.zeros((a.M * a.n // 32 + 64, 2), dtype=torch.int32, device=dev)
    pinfo = torch.empty((256,), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p

    def run(v):
        rc = lib.cs_variant(ctypes.c_int(v), P(X.data_ptr()), ctypes.c_int64(a.n), ctypes.c_int(a.d), ctypes.c_int(a.M),
                            ctypes.c_int(dsub), P(C.data_ptr()), P(base + L["cn"]), P(base + L["img"]),
                            P(base + L["hinit"]), P(base + L["bnd"]), P(base + L["pd"]), P(base + L["bnd2"]),
                            P(codesT.data_ptr()), P(items.data_ptr()), P(counts.data_ptr()), P(pinfo.data_ptr()),
                            P(st))
        assert rc == 0, rc

    run(0)
    torch.cuda.synchronize()
    print(f"M={a.M} dsub={dsub}: codes equal the library: {bool((codesT.t() == ref).all())}", flush=True)
    # interleaved: every round runs each variant once (the clock drifts between rounds)
    times = {v: [] for v in VARIANTS}
    for v in VARIANTS:
        run(v)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        for v in VARIANTS:
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record(); run(v); e_.record()
            torch.cuda.synchronize()
            times[v].append(s_.elapsed_time(e_))
    for v, name in VARIANTS.items():
        t = sorted(times[v])
        print(f"V={v:#10x} {name:44s} median {t[len(t) // 2]:7.3f} ms  min {t[0]:7.3f}", flush=True)


if __name__ == "__main__":
    main()
