"""Shared test setup.

* registers the ``gpu`` marker (tests that need an MI355X; run with ``-m gpu``);
* puts the repo root (for ``oracle``) and the product directory
  ``pathtracker-models_amd`` (for ``ptamd`` / ``models`` / ``utils``, the
  reference-shaped package layout) on ``sys.path``.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "pathtracker-models_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
