"""(method, bpd, D) -> adapter-wrapped quantizer.

Same dispatch as /root/reference/src/haag_vq/benchmarks/method_registry.py:12-61:
PQ / OPQ use B = 8 and M = largest_divisor_leq(D, round(bpd*D) // 8); SQ uses 4 bits for
bpd <= 4.5, 8 for bpd <= 12, else 16; ``rabitq`` routes to the multi-bit Extended RaBitQ
(method_registry_saq.py:45-48).  The SAQ-engine / LVQ / rank-aware research methods are out
of scope of the MI355X build and raise ValueError.
"""

from __future__ import annotations

from haag_vq.benchmarks.quantizer_adapters import FaissQuantizerAdapter

FAISS_METHODS = ("pq", "opq", "sq")
PQ_BITS_PER_SUB = 8


def largest_divisor_leq(D: int, m: int) -> int:
    """Largest divisor of D that is <= m (and >= 1)."""
    m = max(1, min(m, D))
    for cand in range(m, 0, -1):
        if D % cand == 0:
            return cand
    return 1


def _pq_subquantizers(bpd: float, D: int) -> int:
    total_bits = int(round(bpd * D))
    m = max(1, total_bits // PQ_BITS_PER_SUB)
    return largest_divisor_leq(D, m)


def build_faiss_quantizer(method: str, bpd: float, D: int) -> FaissQuantizerAdapter:
    if method == "pq":
        from haag_vq.methods.product_quantization import ProductQuantizer
        return FaissQuantizerAdapter(ProductQuantizer(M=_pq_subquantizers(bpd, D), B=PQ_BITS_PER_SUB))
    if method == "opq":
        from haag_vq.methods.optimized_product_quantization import OptimizedProductQuantizer
        return FaissQuantizerAdapter(OptimizedProductQuantizer(M=_pq_subquantizers(bpd, D), B=PQ_BITS_PER_SUB))
    if method == "sq":
        from haag_vq.methods.scalar_quantization import ScalarQuantizer
        nb = 4 if bpd <= 4.5 else (8 if bpd <= 12 else 16)
        return FaissQuantizerAdapter(ScalarQuantizer(num_bits=nb))
    raise ValueError(f"Unknown faiss method: {method!r}")


SUPPORTED_SAQ_METHODS = ("rabitq",)
SAQ_METHODS = ("saq_paper", "ours", "ours_exact", "rabitq", "lvq",
               "rankaware", "perdim_mse", "rankaware_exact", "perdim_mse_exact")
ALL_METHODS = FAISS_METHODS + SAQ_METHODS


def build_saq_quantizer(method: str, bpd: float, D: int):
    if method == "rabitq":
        from haag_vq.methods.extended_rabitq import ExtendedRaBitQuantizer
        return FaissQuantizerAdapter(ExtendedRaBitQuantizer(num_bits=int(round(bpd))))
    if method in SAQ_METHODS:
        raise ValueError(f"{method!r} is a SAQ-study research method, out of scope of the MI355X build")
    raise ValueError(f"Unknown SAQ-study method: {method!r}")


def build_quantizer(method: str, bpd: float, D: int):
    """Dispatch to the faiss family or the (supported) SAQ-study family."""
    if method in FAISS_METHODS:
        return build_faiss_quantizer(method, bpd=bpd, D=D)
    if method in SAQ_METHODS:
        return build_saq_quantizer(method, bpd=bpd, D=D)
    raise ValueError(f"Unknown method: {method!r}")
