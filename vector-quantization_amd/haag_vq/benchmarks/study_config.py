"""YAML configuration of the quantizer study (the reference's
/root/reference/src/haag_vq/benchmarks/study_config.py:12-36): the dataset block, the
(method, bpd) grid, the recall cut-offs and the chunking knobs of ``run_study``."""

from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List

import yaml

_DEFAULT_KS = (1, 10, 100)


@dataclass
class StudyConfig:
    dataset: Dict[str, Any]
    methods: List[str]
    bpd: List[float]
    ks: List[int] = field(default_factory=lambda: list(_DEFAULT_KS))
    chunk_size: int = 50_000
    mse_sample: int = 100_000
    output_dir: str = "results"


def load_study_config(path: str | Path) -> StudyConfig:
    """Reads the YAML file with ``yaml.safe_load`` (nothing in the file is executed); missing
    optional keys take the dataclass defaults, as upstream."""
    raw = yaml.safe_load(Path(path).read_text(encoding="utf-8")) or {}
    for key in ("dataset", "methods", "bpd"):
        if key not in raw:
            raise KeyError(key)
    opt = {
        "ks": [int(k) for k in raw.get("ks", _DEFAULT_KS)],
        "chunk_size": int(raw.get("chunk_size", 50_000)),
        "mse_sample": int(raw.get("mse_sample", 100_000)),
        "output_dir": str(raw.get("output_dir", "results")),
    }
    return StudyConfig(dataset=raw["dataset"], methods=list(raw["methods"]), bpd=list(raw["bpd"]), **opt)
