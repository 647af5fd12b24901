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


def icy_stencil_rect(W, H, p_slip):
    """STENCIL5 row form [A = 4, 5, S] of an IcyGridWorld on a W x H grid: the
    square builder's per-state rules (gridworld.py:177-248) with separate
    widths and heights (no reference counterpart: the reference's worlds are
    square; used to exercise rectangular tilings)."""
    S = W * H
    s = np.arange(S)
    x, y = s % W, s // W
    na = 4
    p_int, p_nb = 1.0 - p_slip + p_slip / na, p_slip / na
    corner = ((x == 0) | (x == W - 1)) & ((y == 0) | (y == H - 1))
    edge = (x == 0) | (x == W - 1) | (y == 0) | (y == H - 1)
    dirs = [(1, 0), (-1, 0), (0, 1), (0, -1)]            # actions (gridworld.py:47), also slots 1..4
    rv = np.zeros((na, 5, S))
    for a, (ax, ay) in enumerate(dirs):
        for k, (dx, dy) in enumerate(dirs):
            ok = (x + dx >= 0) & (x + dx < W) & (y + dy >= 0) & (y + dy < H)
            rv[a, k + 1] = np.where(ok, p_int if (dx, dy) == (ax, ay) else p_nb, 0.0)
        over = ~((x + ax >= 0) & (x + ax < W) & (y + ay >= 0) & (y + ay < H))
        stay = np.zeros(S)
        stay[over & corner] = 1.0 - p_slip + 2.0 * p_slip / na
        stay[over & ~corner] = 1.0 - p_slip + p_slip / na
        stay[~over & corner] = 2.0 * p_slip / na
        stay[~over & ~corner & edge] = p_slip / na
        rv[a, 0] = stay
    return rv
