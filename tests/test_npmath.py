"""numpy's float64 exp / log (soft VI's softmax, maxent.py:260-276, and its
policy, maxent.py:341), restated in the oracle (oracle/blas_order.c) and on the
device (np_exp / np_log, csrc/common.h).  Here, without a GPU:

* the fixture (tests/golden/npmath.npz, tools/gen_npmath.py) is numpy's own
  output on this host when numpy dispatches to the same AVX512_SKX loops;
* the oracle's restatement equals it bit for bit on the ~116k sampled
  arguments (ranges, rare-path edges, special values) and on the 2 x 10^6
  hashed ones;
* the rcp14 thresholds in the device and oracle sources are the fixture's
  (measured by tools/npmath_rcp14.c on an AVX-512 host);
* the ABI entry irlmx_numpy_math validates its arguments.
The device side is tests/test_gpu_npmath.py."""
import ctypes
import hashlib
import os
import re
import sys

import numpy as np
import pytest

import maxent_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gen_npmath import big_args  # noqa: E402

Z = np.load(os.path.join(ROOT, "tests", "golden", "npmath.npz"))


@pytest.fixture(scope="module", autouse=True)
def built():
    import __graft_entry__ as g
    g.build_oracle()


def same_bits(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    return (a.view(np.uint64) == b.view(np.uint64)) | both_nan


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def test_fixture_is_this_hosts_numpy():
    feats = np._core._multiarray_umath.__cpu_features__
    if np.__version__ != str(Z["numpy_version"]) or not feats.get("AVX512_SKX"):
        pytest.skip(f"numpy {np.__version__} / no AVX512_SKX: another exp / log implementation")
    with np.errstate(all="ignore"):
        assert same_bits(np.exp(Z["x_exp"]), Z["y_exp"]).all()
        assert same_bits(np.log(Z["x_log"]), Z["y_log"]).all()


@pytest.mark.parametrize("fn,key", [(O.numpy_exp_restated, "exp"), (O.numpy_log_restated, "log")])
def test_oracle_restatement_bit_exact(fn, key):
    ok = same_bits(fn(Z["x_" + key]), Z["y_" + key])
    bad = np.nonzero(~ok)[0]
    assert ok.all(), f"{len(bad)} mismatches, first x = {Z['x_' + key][bad[:3]]}"


def test_oracle_restatement_hashed_sets():
    xe, xl = big_args(int(Z["big_seed"]), int(Z["big_n"]))
    assert sha(O.numpy_exp_restated(xe)) == str(Z["big_sha_exp"])
    assert sha(O.numpy_log_restated(xl)) == str(Z["big_sha_log"])


def test_restated_differs_from_correctly_rounded():
    """The point of the restatement: numpy's exp is not libm's (one ulp apart on
    a few percent of arguments), so ocml or glibc would not do."""
    import math
    x = Z["x_exp"][20:10020]
    libm = np.array([math.exp(v) for v in x])
    assert (~same_bits(libm, Z["y_exp"][20:10020])).sum() > 100


def test_rcp_thresholds_in_sources():
    steps = [int(t) for t in Z["rcp_steps"]]
    dev = open(os.path.join(ROOT, "irl-maxent_amd", "csrc", "common.h")).read()
    got = [int(t) for t in re.findall(r"\(u >= (\d+)u\)", dev)]
    assert got == steps
    orc = open(os.path.join(ROOT, "oracle", "blas_order.c")).read()
    body = re.search(r"kRcpSteps\[16\] = \{([^}]*)\}", orc).group(1)
    assert [int(t) for t in re.findall(r"(\d+)u", body)] == steps


def test_rcp_bucket_table_equals_thresholds():
    """The device's default reciprocal count (IRLMX_NPMATH_BUCKET: one 256-entry
    table read) is the 16-threshold count for every 16-bit mantissa prefix."""
    dev = open(os.path.join(ROOT, "irl-maxent_amd", "csrc", "common.h")).read()
    body = dev[dev.index("unsigned rcp[256];"):]
    body = body[body.index("{{"):body.index("}};")]
    ent = [int(t, 16) for t in re.findall(r"0x([0-9a-f]+)u", body.split("},")[-1])]
    assert len(ent) == 256
    steps = np.array([int(t) for t in Z["rcp_steps"]])
    u = np.arange(65536)
    e = np.array(ent)[u >> 8]
    nd = (e & 0xFF) + ((u & 255) >= (e >> 8))
    assert np.array_equal(nd, (u[:, None] >= steps[None, :]).sum(axis=1))


def test_numpy_math_arguments():
    import irlmx._lib as L
    lib = L.load()
    x = np.zeros(4)
    assert lib.irlmx_numpy_math(2, x.ctypes.data, x.ctypes.data, 4, None) == -1
    assert "unknown op 2" in lib.irlmx_last_error().decode()
    assert lib.irlmx_numpy_math(0, x.ctypes.data, x.ctypes.data, -1, None) == -1
    assert lib.irlmx_numpy_math(1, None, x.ctypes.data, 4, None) == -1
    assert lib.irlmx_numpy_math(0, None, None, 0, None) == 0
