"""The drop-ins' numpy-order scope per op (irlmx.ops.numpy_order_default; CPU,
no device call): value iteration and soft VI run in numpy's order on every
model the kernels cover up to 4096 states (config 2's 64x64), the backward and
the forward up to 1024; DENSE tables 64 except value iteration; the
environment overrides; batches and uncovered sizes never."""

import types

import pytest


@pytest.fixture(scope="module")
def ops():
    import __graft_entry__ as g
    g.build()
    from irlmx import ops
    return ops


def model(ops, S, layout="stencil", batch=1, k_col=5):
    from irlmx import _lib
    lay = {"stencil": _lib.LAYOUT_STENCIL5, "ell": _lib.LAYOUT_ELL, "dense": _lib.LAYOUT_DENSE}[layout]
    return types.SimpleNamespace(n_states=S, layout=lay, batch=batch, k_col=k_col)


def test_default_caps(ops, monkeypatch):
    for k in ("IRLMX_NUMPY_ORDER", "IRLMX_NUMPY_ORDER_MAX", "IRLMX_NUMPY_ORDER_DENSE_MAX", "IRLMX_NUMPY_ORDER_BWD_MAX",
              "IRLMX_NUMPY_ORDER_FWD_MAX", "IRLMX_NUMPY_ORDER_SOFT_MAX", "IRLMX_NUMPY_ORDER_VI_MAX"):
        monkeypatch.delenv(k, raising=False)
    c2 = model(ops, 4096)                       # config 2: 64x64
    assert ops.numpy_order_default(c2, "value_iteration") and ops.numpy_order_default(c2, "soft_backward")
    assert not ops.numpy_order_default(c2, "backward") and not ops.numpy_order_default(c2, "forward")
    small = model(ops, 1024)                    # 32x32
    assert all(ops.numpy_order_default(small, op) for op in ("backward", "forward", "soft_backward", "value_iteration"))
    assert not ops.numpy_order_default(model(ops, 16384), "value_iteration")        # beyond the kernels
    assert not ops.numpy_order_default(model(ops, 4094), "value_iteration")         # S % 4 == 2
    assert not ops.numpy_order_default(model(ops, 1024, batch=2), "value_iteration")  # batches: tiled shapes
    dense = model(ops, 1024, "dense")
    assert ops.numpy_order_default(dense, "value_iteration")
    assert not ops.numpy_order_default(dense, "soft_backward") and not ops.numpy_order_default(dense, "backward")
    assert ops.numpy_order_default(model(ops, 64, "dense"), "backward")
    assert not ops.numpy_order_default(model(ops, 1024, "ell", k_col=40), "forward")  # ELL column form > 32 slots


def test_environment_overrides(ops, monkeypatch):
    c2 = model(ops, 4096)
    monkeypatch.setenv("IRLMX_NUMPY_ORDER_MAX", "4096")
    assert ops.numpy_order_default(c2, "backward") and ops.numpy_order_default(c2, "forward")
    monkeypatch.setenv("IRLMX_NUMPY_ORDER_FWD_MAX", "1024")
    assert not ops.numpy_order_default(c2, "forward") and ops.numpy_order_default(c2, "backward")
    monkeypatch.delenv("IRLMX_NUMPY_ORDER_MAX")
    monkeypatch.setenv("IRLMX_NUMPY_ORDER_VI_MAX", "1024")
    assert not ops.numpy_order_default(c2, "value_iteration") and ops.numpy_order_default(c2, "soft_backward")
    monkeypatch.setenv("IRLMX_NUMPY_ORDER_DENSE_MAX", "2048")
    assert ops.numpy_order_default(model(ops, 1024, "dense"), "soft_backward")
    monkeypatch.setenv("IRLMX_NUMPY_ORDER", "0")
    assert not any(ops.numpy_order_default(model(ops, 64), op)
                   for op in ("backward", "forward", "soft_backward", "value_iteration"))
