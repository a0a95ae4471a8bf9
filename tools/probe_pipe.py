"""Interleaved A/B of mivq_pq_encode slice configurations (one library, one process, same data).

usage: python tools/probe_pipe.py --n 1000000 --cfg base:PIPE=0 --cfg s2:SLICES=2 ...
Each --cfg is NAME:VAR=VAL[,VAR=VAL] over the profiling variables MIVQ_PQ_PIPE,
MIVQ_PQ_SLICES, MIVQ_PQ_SLICE_ROWS (set in the process environment before each call; the
library reads them per call).  Prints per-call medians (HIP events on the caller's stream,
which the call joins) and checks every configuration's codes against the first one's.
"""
import argparse
import ctypes
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from bench import synth  # noqa: E402

KEYS = ("MIVQ_PQ_PIPE", "MIVQ_PQ_SLICES", "MIVQ_PQ_SLICE_ROWS")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--data", default="gaussian")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--cfg", action="append", required=True)
    a = ap.parse_args()
    cfgs = []
    for c in a.cfg:
        name, _, rest = c.partition(":")
        env = {}
        for kv in filter(None, rest.split(",")):
            k, v = kv.split("=")
            env["MIVQ_PQ_" + k] = v
        cfgs.append((name, env))
    dev = _native.require_device()
    lib = _native.load_library()
    X = synth(a.n, a.d, 0, dev, kind=a.data)
    C = train_pq(X[:65536], a.M, 8, niter=25, seed=1234).contiguous()
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p
    prep = torch.empty(lib.mivq_pq_prep_bytes(a.d, a.M, 8), dtype=torch.uint8, device=dev)
    assert lib.mivq_pq_prepare(P(C.data_ptr()), a.d, a.M, 8, P(prep.data_ptr()), P(st)) == 0
    ws = torch.empty(lib.mivq_pq_encode_workspace_bytes(a.n, a.d, a.M, 8), dtype=torch.uint8, device=dev)
    outs = {name: torch.empty((a.n, a.M), dtype=torch.uint8, device=dev) for name, _ in cfgs}

    def run(name, env, out=None):
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        o = outs[name] if out is None else out
        rc = lib.mivq_pq_encode(P(X.data_ptr()), a.n, a.d, a.M, 8, P(C.data_ptr()), P(prep.data_ptr()),
                                P(ws.data_ptr()), ws.numel(), P(o.data_ptr()), 0, P(st))
        assert rc == 0, (rc, lib.mivq_last_error())

    for name, env in cfgs:
        run(name, env)
    torch.cuda.synchronize()
    ref = outs[cfgs[0][0]]
    for name, _ in cfgs:
        print(f"{name}: codes identical to {cfgs[0][0]}: {bool(torch.equal(outs[name], ref))}", flush=True)
    # settle the clock, then interleave
    for _ in range(3):
        for name, env in cfgs:
            run(name, env)
    torch.cuda.synchronize()
    res = {name: [] for name, _ in cfgs}
    for _ in range(a.reps):
        for name, env in cfgs:
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            run(name, env)
            e_.record()
            torch.cuda.synchronize()
            res[name].append(s_.elapsed_time(e_))
    gb = a.n * (4 * a.d + a.M) / 1e9
    for name, _ in cfgs:
        t = sorted(res[name])
        med = t[len(t) // 2]
        print(f"PIPE {name:10s} median {med:.3f} ms  min {t[0]:.3f}  max {t[-1]:.3f}  "
              f"= {gb / med / 8.0:.3f} of 8 TB/s", flush=True)
    for name, env in cfgs:  # back to back (what the bench's timed loop sees)
        for _ in range(2):
            run(name, env)
        s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s_.record()
        for _ in range(10):
            run(name, env)
        e_.record()
        torch.cuda.synchronize()
        ms = s_.elapsed_time(e_) / 10
        print(f"B2B {name:10s} {ms:.3f} ms/call = {gb / ms / 8.0:.3f} of 8 TB/s", flush=True)
    for name, _ in cfgs:
        assert torch.equal(outs[name], ref), name


if __name__ == "__main__":
    main()
