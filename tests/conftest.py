"""Test configuration: import paths, the ``gpu`` marker and shared fixtures.

CPU tests (``-m "not gpu"``) cover the oracle against the reference-derived
golden vectors, the host logic, the C-ABI exports and the distributed logic
(gloo).  GPU tests (``-m gpu``) are the parity tests proper: they call the HIP
library through the C ABI and compare with the oracle / golden fixtures.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "gnn-fraud-detection_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); runs the libgfd.so kernels")
    config.addinivalue_line("markers", "slow: long-running (full-size) test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]
    return get
