"""The device's numpy exp / log (np_exp / np_log, csrc/common.h; soft VI's
softmax and policy, maxent.py:260-276 / 341) against numpy's own results
(tests/golden/npmath.npz, tools/gen_npmath.py: numpy 2.2.6's AVX512_SKX loops
on the fixture host), through the C ABI's irlmx_numpy_math: bit for bit on
the ~116k sampled arguments (soft VI's ranges, the full ranges, rare-path
edges, specials) and, by sha256, on 2 x 10^6 more."""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gen_npmath import big_args  # noqa: E402

pytestmark = pytest.mark.gpu
Z = np.load(os.path.join(ROOT, "tests", "golden", "npmath.npz"))


@pytest.fixture(scope="module")
def dev():
    import irlmx
    return irlmx.require_device()


def device_math(op, x, dev):
    import irlmx._lib as L
    lib = L.load()
    xd = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=dev)
    yd = torch.empty_like(xd)
    L.check(lib.irlmx_numpy_math(op, xd.data_ptr(), yd.data_ptr(), xd.numel(), L.stream_ptr(dev)), "numpy_math")
    return yd.cpu().numpy()


def same_bits(a, b):
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


@pytest.mark.parametrize("op,key", [(0, "exp"), (1, "log")])
def test_device_numpy_math_bit_exact(dev, op, key):
    x, want = Z["x_" + key], Z["y_" + key]
    got = device_math(op, x, dev)
    ok = same_bits(got, want)
    bad = np.flatnonzero(~ok)
    assert ok.all(), (key, len(bad), [(float(x[i]).hex(), float(got[i]).hex(), float(want[i]).hex()) for i in bad[:4]])


def test_device_numpy_math_hashed_sets(dev):
    xe, xl = big_args(int(Z["big_seed"]), int(Z["big_n"]))
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert sha(device_math(0, xe, dev)) == str(Z["big_sha_exp"])
    assert sha(device_math(1, xl, dev)) == str(Z["big_sha_log"])
