"""Interleaved timing of mivq_adc_search: the filtered path vs the fp32 scan (flag MIVQ_ADC_FORCE_EXACT),
same process and data; checks ids / distances identical.

usage: python tools/probe_adc.py [--n 1000000] [--nq 1000] [--M 16] [--k 10] [--reps 10] [--data gaussian]
Codes are the PQ encode of synthetic rows (bench.synth) with k-means codebooks, as in bench.py.
"""
import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vector-quantization_amd"))
sys.path.insert(0, str(ROOT))
from haag_vq import _native  # noqa: E402
from haag_vq.methods._kmeans import train_pq  # noqa: E402
from bench import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--M", type=int, default=16)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--data", default="gaussian")
    a = ap.parse_args()
    dev = _native.require_device()
    X = synth(a.n, a.d, 0, dev, kind=a.data)
    C = train_pq(X[:65536], a.M, 8, niter=25, seed=1234).contiguous()
    prep = _native.pq_prepare(C, 8)
    codes = _native.pq_encode(X, C, prep, 8)
    del X
    Q = synth(a.nq, a.d, 7, dev, kind=a.data)
    lut = _native.adc_lut(Q, C, 8, _native.METRIC_L2)

    def run(exact):
        return _native.adc_search(lut, codes, a.k, 8, flags=_native.ADC_FORCE_EXACT if exact else _native.ADC_AUTO)

    fd, fi = run(False)
    ed, ei = run(True)
    torch.cuda.synchronize()
    same = bool(torch.equal(fd, ed) and torch.equal(fi, ei))
    print(f"identical: {same}", flush=True)
    res = {False: [], True: []}
    for _ in range(a.reps):
        for ex in (False, True):
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            run(ex)
            e_.record()
            torch.cuda.synchronize()
            res[ex].append(s_.elapsed_time(e_))
    for ex in (False, True):
        t = sorted(res[ex])
        med = t[len(t) // 2]
        lds = a.nq * a.n * a.M * 4 / (med * 1e-3) / 1e12
        print(f"ADC {'fp32 scan' if ex else 'filtered '} nq={a.nq} n={a.n} M={a.M} k={a.k}: median {med:.3f} ms "
              f"min {t[0]:.3f} = {a.nq / med * 1e3:.0f} q/s, {lds:.1f} TB/s of fp32-LUT reads = {lds / 157.3:.3f} of LDS peak",
              flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
