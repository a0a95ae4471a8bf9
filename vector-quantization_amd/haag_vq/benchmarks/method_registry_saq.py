"""Registry of the SAQ-study methods — module path of
/root/reference/src/haag_vq/benchmarks/method_registry_saq.py:1-74.

Callers import ``build_saq_quantizer`` / ``SAQ_METHODS`` from here (the reference's
``quantizer_study`` and its tests do).  Of these methods only ``rabitq`` (the multi-bit
Extended RaBitQ, :45-48) is on the MI355X path; the SAQ-engine, LVQ and rank-aware research
methods are out of scope and raise ValueError.  The implementation lives in
``method_registry`` (one dispatch table for both families).
"""

from haag_vq.benchmarks.method_registry import SAQ_METHODS, SUPPORTED_SAQ_METHODS, build_saq_quantizer

__all__ = ["SAQ_METHODS", "SUPPORTED_SAQ_METHODS", "build_saq_quantizer"]
