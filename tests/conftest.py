"""Shared test setup.

Markers: `gpu` = needs a HIP device (MI355X) and runs the native kernels through the C-ABI.
Everything else runs on CPU (oracle vs golden vectors, host logic, ABI exports, gloo).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "02-visualodometry_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def vo():
    from picp_amd.vo_data import VOData
    return VOData()


@pytest.fixture(scope="session")
def native():
    """The HIP library on a real device; fails (never skips silently) on a GPU run."""
    import picp_amd
    picp_amd.lib()
    n = picp_amd.device_count()
    assert n >= 1, "no HIP device visible"
    return picp_amd
