from .faiss_ivfpq_index import FaissIvfPqIndex
from .flat_quantized_index import FlatQuantizedIndex, FlatADCIndex, search_codes
from .rabitq_index import RaBitQIndex

__all__ = ["FaissIvfPqIndex", "FlatQuantizedIndex", "FlatADCIndex", "RaBitQIndex", "search_codes"]
