import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "fhe-icp_amd"
for p in (str(PKG), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libfheicp.so")
    config.addinivalue_line("markers", "slow: long-running CPU oracle test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import tfhe_ref
    tfhe_ref.build()
    return tfhe_ref


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def need_gpu():
    if not gpu_available():
        pytest.skip("no GPU")
    return True
