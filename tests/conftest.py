"""Test configuration: the ``gpu`` marker and import paths.

``-m "not gpu"``: oracle vs golden vectors, host planner, C-ABI exports, gloo
multi-process plumbing (CPU only).  ``-m gpu``: HIP parity tests through the C-ABI.
"""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "radio-pulsar-utils_amd")
for p in (PKG_DIR, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the HIP library")


@pytest.fixture(scope="session")
def golden():
    with np.load(os.path.join(GOLDEN_DIR, "golden.npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    meta = json.load(open(os.path.join(GOLDEN_DIR, "golden.json")))
    return arrays, meta


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    return torch.device("cuda", 0)
