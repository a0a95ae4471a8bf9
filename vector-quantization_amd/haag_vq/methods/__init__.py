"""Quantizers of the MI355X build (module paths mirror /root/reference/src/haag_vq/methods)."""

from .base_quantizer import BaseQuantizer
from .base_search_index import BaseSearchIndex

__all__ = ["BaseQuantizer", "BaseSearchIndex"]
