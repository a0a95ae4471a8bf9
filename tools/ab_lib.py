"""Interleaved A/B of mivq_pq_encode between two builds of libmivq.so (same process, same data).

usage: python tools/ab_lib.py OTHER.so [--what encode|adc|lut] [--n 1000000] [--d 1536] [--M 16]
                              [--data gaussian] [--reps 10] [--nq 1000] [--k 10]
The in-tree library (vector-quantization_amd/lib/libmivq.so) is "this"; OTHER.so is e.g. a
build of the previous commit (git stash; make; cp lib/libmivq.so /tmp/old.so; git stash pop).
Prints per-call medians of alternating single calls (HIP events) and back-to-back rates, and
checks that both builds emit identical codes (--what adc: mivq_adc_search over the encoded
rows, identical ids and distances).
"""
import argparse
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from bench import synth  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in _native.SIGNATURES.items():
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("other")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--data", default="gaussian")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--what", choices=("encode", "adc", "lut"), default="encode")
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    a = ap.parse_args()
    dev = _native.require_device()
    libs = {"this": bind(_native.LIB_PATH), "other": bind(a.other if Path(a.other).is_absolute() else ROOT / a.other)}
    X = synth(a.n, a.d, 0, dev, kind=a.data)
    C = train_pq(X[:65536], a.M, 8, niter=25, seed=1234).contiguous()
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p
    state = {}
    for k, lb in libs.items():
        prep = torch.empty(lb.mivq_pq_prep_bytes(a.d, a.M, 8), dtype=torch.uint8, device=dev)
        assert lb.mivq_pq_prepare(P(C.data_ptr()), a.d, a.M, 8, P(prep.data_ptr()), P(st)) == 0
        nb = lb.mivq_pq_encode_workspace_bytes(a.n, a.d, a.M, 8)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        out = torch.empty((a.n, a.M), dtype=torch.uint8, device=dev)
        state[k] = (prep, ws, out)

    def run_encode(k):
        lb = libs[k]
        prep, ws, out = state[k]
        rc = lb.mivq_pq_encode(P(X.data_ptr()), a.n, a.d, a.M, 8, P(C.data_ptr()), P(prep.data_ptr()),
                               P(ws.data_ptr()), ws.numel(), P(out.data_ptr()), 0, P(st))
        assert rc == 0, rc

    run = run_encode
    for k in libs:
        run_encode(k)
    torch.cuda.synchronize()
    same = bool(torch.equal(state["this"][2], state["other"][2]))
    if a.what == "lut":  # mivq_adc_lut alone: the LUTs of nq queries, compared bit for bit
        Q = synth(a.nq, a.d, 7, dev, kind=a.data)
        luts = {k: torch.empty((a.nq, a.M, 256), dtype=torch.float32, device=dev) for k in libs}

        def run_lut(k):
            rc = libs[k].mivq_adc_lut(P(Q.data_ptr()), a.nq, a.d, a.M, 8, P(C.data_ptr()), 1, P(luts[k].data_ptr()), P(st))
            assert rc == 0, rc

        run = run_lut
        for k in libs:
            run_lut(k)
        torch.cuda.synchronize()
        same = bool(torch.equal(luts["this"], luts["other"]))
    if a.what == "adc":
        codes = state["this"][2]
        Q = synth(a.nq, a.d, 7, dev, kind=a.data)
        lut = torch.empty((a.nq, a.M, 256), dtype=torch.float32, device=dev)
        assert libs["this"].mivq_adc_lut(P(Q.data_ptr()), a.nq, a.d, a.M, 8, P(C.data_ptr()), 1, P(lut.data_ptr()),
                                         P(st)) == 0
        adc = {}
        for k, lb in libs.items():
            nb = lb.mivq_adc_search_workspace_bytes(a.nq, a.n, a.M, 8, a.k)
            adc[k] = (torch.empty(max(nb, 256), dtype=torch.uint8, device=dev),
                      torch.empty((a.nq, a.k), dtype=torch.float32, device=dev),
                      torch.empty((a.nq, a.k), dtype=torch.int32, device=dev))

        def run_adc(k):
            ws, od, oi = adc[k]
            rc = libs[k].mivq_adc_search(P(lut.data_ptr()), a.nq, P(codes.data_ptr()), a.n, a.M, 8, a.k, 0,
                                         P(ws.data_ptr()), ws.numel(), P(od.data_ptr()), P(oi.data_ptr()), 0, P(st))
            assert rc == 0, rc

        run = run_adc
        for k in libs:
            run_adc(k)
        torch.cuda.synchronize()
        same = bool(torch.equal(adc["this"][1], adc["other"][1]) and torch.equal(adc["this"][2], adc["other"][2]))
    print(f"{a.what}: outputs identical: {same}", flush=True)
    res = {k: [] for k in libs}
    for _ in range(a.reps * 3):
        for k in libs:
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record(); run(k); e_.record()
            torch.cuda.synchronize()
            res[k].append(s_.elapsed_time(e_))
    for k in libs:
        t = sorted(res[k])
        print(f"AB {k}: median {t[len(t) // 2]:.3f} ms  min {t[0]:.3f}  max {t[-1]:.3f}", flush=True)
    for rnd in range(2):
        for k in libs:
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                run(k)
            s_.record()
            for _ in range(20):
                run(k)
            e_.record()
            torch.cuda.synchronize()
            ms = s_.elapsed_time(e_) / 20
            if a.what == "encode":
                gbs = a.n * (4 * a.d + a.M) / (ms * 1e-3) / 1e9
                print(f"AB {k} round {rnd}: back-to-back {ms:.3f} ms/call = {gbs / 8000:.3f} of 8 TB/s", flush=True)
            else:
                print(f"AB {k} round {rnd}: back-to-back {ms:.3f} ms/call = {a.nq / ms * 1e3:.0f} queries/s", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
