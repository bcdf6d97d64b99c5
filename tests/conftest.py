"""Test configuration: import paths, the `gpu` marker, and in-tree builds.

-m "not gpu": oracle vs golden vectors, host logic, ABI surface (runs in the build
container, no GPU).  -m gpu: parity of the HIP kernels (through the C ABI) vs the oracle.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "real-time_fraud_detection_system_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def _ensure_built():
    lib = os.path.join(PKG, "fdx", "libfdx.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(PKG, "csrc")])
    olib = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(olib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)

    return load


@pytest.fixture(scope="session")
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return torch.device("cuda", 0)
