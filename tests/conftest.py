"""Test configuration: `gpu` marker, import paths, shared fixtures.

* ``-m "not gpu"`` (CPU container): oracle vs golden fixtures / KATs, host logic, and the
  C-ABI library loads and exports every symbol of include/mivq.h.
* ``-m gpu`` (MI355X box): parity of every HIP entry point against the oracle.
"""

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "vector-quantization_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the parity tests")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # noqa: E402  (test infrastructure only)

    O.build()
    return O


@pytest.fixture(scope="session")
def golden_dir():
    return ROOT / "tests" / "golden"


@pytest.fixture(scope="session")
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from haag_vq import _native

    return _native.require_device()
