"""Metric enum shared with faiss (same values as /root/reference/src/haag_vq/utils/faiss_utils.py:3-17)."""

from enum import IntEnum


class MetricType(IntEnum):
    INNER_PRODUCT = 0  # maximum inner product search
    L2 = 1             # squared L2 search
    L1 = 2
    Linf = 3
    Lp = 4
    Canberra = 20
    BrayCurtis = 21
    JensenShannon = 22
    Jaccard = 23
    NaNEuclidean = 24
    GOWER = 25
