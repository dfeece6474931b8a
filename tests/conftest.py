import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / 'marl-factory-grid_amd', ROOT / 'oracle', ROOT / 'tests'):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device')


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
