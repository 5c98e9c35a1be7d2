"""Shared test setup.

* ``gpu`` marker: needs a real MI355X (run with ``-m gpu``); those tests call
  libggs.so through its C ABI and compare against the oracle / golden fixtures.
* Everything else runs on CPU: the oracle against the reference-generated
  golden vectors, host logic, the C-ABI surface (load + exports, no compute),
  and the multi-rank path over gloo.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "genetic-gaussian-splats_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: larger parity sizes")


def load_golden(name: str):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden
