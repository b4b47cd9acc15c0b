import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
import stereoalgorithms_amd  # noqa: E402,F401  (sets HIP runtime env before torch initialises the GPU)

FIXTURES = ROOT / "tests" / "fixtures"


def pytest_configure(config):
    # keep test scratch files (tmp_path) inside the repository's git-ignored build/ directory
    if getattr(config.option, "basetemp", None) is None:
        (ROOT / "build").mkdir(exist_ok=True)
        config.option.basetemp = str(ROOT / "build" / "pytest-tmp")
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the native library")
    config.addinivalue_line("markers", "slow: long-running")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def fixtures_dir():
    return FIXTURES
