from .faiss_utils import MetricType

__all__ = ["MetricType"]
