"""Test configuration: `-m gpu` tests need an MI355X (HIP); everything else runs on CPU."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "helpers"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and the built HIP extension")


@pytest.fixture(scope="session")
def model():
    from h12env.model import build_model

    return build_model()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (run with -m 'not gpu' on CPU hosts)")
    from h12env._abi import load_library

    load_library()  # fails loudly if the HIP extension is missing
    return torch.device("cuda:0")
