"""Shared pytest configuration.

* registers the ``gpu`` marker (tests that need an MI355X; run with ``-m gpu``)
* puts the product package directory (``irl-maxent_amd/``) and the oracle on
  ``sys.path``; the oracle is imported by tests only, as the checker.
"""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "irl-maxent_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")

for p in (PKG_DIR, ORACLE_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def unpack_trajectories(flat, lens):
    """Rebuild reference-style trajectories from the packed fixture arrays."""
    from maxent_oracle import Trajectory
    out, o = [], 0
    for n in lens:
        out.append(Trajectory([tuple(int(v) for v in row) for row in flat[o:o + n]]))
        o += n
    return out


@pytest.fixture(scope="session")
def golden():
    return load_golden
