"""Shared pytest setup: marker registration, import paths, fixtures.

`-m "not gpu"` tests run anywhere (oracle vs golden vectors, host logic, ABI symbol
table, gloo multi-process); `-m gpu` tests drive libmqhip.so on an MI355X through the
C ABI and compare against the oracle."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "mediquery-rag_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libmqhip.so kernels)")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session")
def corpus_docs():
    import json
    with open(os.path.join(GOLDEN, "corpus_docs.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def require_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU test selected but no GPU is visible")
    return True


def rng(seed=0):
    return np.random.default_rng(seed)
