from .distortion import compute_distortion
from .performance import measure_qps, time_compress, time_decompress
from .recall import evaluate_recall

__all__ = ["compute_distortion", "evaluate_recall", "measure_qps", "time_compress", "time_decompress"]
