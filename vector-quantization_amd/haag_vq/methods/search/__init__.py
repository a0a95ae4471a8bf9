from .faiss_ivfpq_index import FaissIvfPqIndex
from .flat_quantized_index import FlatQuantizedIndex, FlatADCIndex, search_codes

__all__ = ["FaissIvfPqIndex", "FlatQuantizedIndex", "FlatADCIndex", "search_codes"]
