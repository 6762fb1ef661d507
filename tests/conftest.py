import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "audio-analysis_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libaa.so on cuda:0)")


@pytest.fixture(scope="session")
def model_root(tmp_path_factory):
    """Seeded build-defined model1/2/3 directories (tools/make_models.py)."""
    from tools.make_models import make_ensemble
    root = tmp_path_factory.mktemp("models")
    make_ensemble(root)
    return root


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
