"""CPU-side checks of the C ABI: the library loads and exports every symbol
include/irlmx.h declares, and the ctypes binding covers all of them.  No
compute call is made (no GPU here)."""

import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "irlmx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(irlmx_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    from irlmx import _lib
    return _lib.load()


def test_header_symbols_exported(lib):
    names = _declared()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n


def test_binding_covers_header(lib):
    from irlmx import _lib
    assert sorted(_lib.SIGNATURES) == _declared()
    assert lib.irlmx_abi_version() == 1


def test_struct_layout_matches_header():
    import ctypes
    from irlmx import _lib
    # 10 int32 then 4 pointers, as declared in irlmx_mdp
    assert ctypes.sizeof(_lib.MDPStruct) == 10 * 4 + 4 * 8
    assert _lib.MDPStruct.row_val.offset == 40


def test_ops_fail_loudly_without_device(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    import irlmx
    with pytest.raises(RuntimeError, match="no HIP device"):
        irlmx.DeviceMDP.icy_gridworld(5, 0.2)
