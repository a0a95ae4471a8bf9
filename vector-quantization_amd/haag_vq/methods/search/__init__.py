from .flat_quantized_index import FlatQuantizedIndex, FlatADCIndex, search_codes

__all__ = ["FlatQuantizedIndex", "FlatADCIndex", "search_codes"]
