"""Failure paths of the persistent shapes that need a device (cluster.hip).

* Co-residency rejection (cluster_run): a plan whose workgroups cannot all be
  resident at once is refused with IRLMX_EINVAL before launch.  Forced by
  letting the planner believe in more CUs than the device has
  (IRLMX_PLAN_CUS).
* Exchange timeout: one workgroup leaves right after the co-residency
  rendezvous (IRLMX_TEST_DROP_TILE) with a shortened exchange limit
  (IRLMX_TEST_EXCHANGE_TIMEOUT_MS), so its neighbours' granule polls time out.
  The call is rerun on the per-sweep shape -- bit-identical results, counted in
  irlmx_counters' rerun_timeout -- or, with IRLMX_STRICT_EXCHANGE=1, fails
  with IRLMX_EHIP and the timeout message.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

B = 4


@pytest.fixture(scope="module")
def dev():
    import __graft_entry__ as g
    g.build()
    import irlmx
    return irlmx.require_device()


def make_world(dev, monkeypatch, size):
    from irlmx import DeviceMDP, ops
    for k in ("IRLMX_PLAN_CUS", "IRLMX_TEST_DROP_TILE", "IRLMX_TEST_EXCHANGE_TIMEOUT_MS", "IRLMX_STRICT_EXCHANGE",
              "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
        monkeypatch.delenv(k, raising=False)
    S = size * size
    mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
    rng = np.random.default_rng(4)
    r = rng.uniform(0.0, 1.0, (B, S))
    term = ops.terminal_mask([S - 1], S, batch=B, device=dev)
    p0 = np.zeros((B, S))
    p0[:, 0] = 1.0
    return mdp, r, term, p0


@pytest.fixture
def world(dev, monkeypatch):
    return make_world(dev, monkeypatch, 64)


@pytest.fixture
def world128(dev, monkeypatch):
    """128x128: several tiles per instance in both passes, so every tile exchanges halos."""
    return make_world(dev, monkeypatch, 128)


def test_coresidency_rejection(world, monkeypatch):
    from irlmx import _lib, ops
    SIZE = 64
    mdp, r, term, p0 = world
    assert ops.execution_plan(mdp, "backward")["shape"] == "cluster"
    monkeypatch.setenv("IRLMX_CLUSTER_R", "4")      # 16 tiles per instance
    monkeypatch.setenv("IRLMX_CLUSTER_G", "2")
    # 72 instances x 16 tiles = 1,152 workgroups: more than any CU count x the at
    # most 4 resident 512-thread workgroups per CU (32 waves) of this device
    n = 72
    big = mdp.take(np.arange(B).repeat(n // B))
    monkeypatch.setenv("IRLMX_PLAN_CUS", "16384")  # planner: 1,024 instances per launch fit
    plan = ops.execution_plan(big, "backward")
    assert plan["C"] == 16 and plan["per_launch"] == n, plan
    n_cus = torch.cuda.get_device_properties(big.device).multi_processor_count
    assert 16 * n > 4 * n_cus
    for call in (lambda: ops.backward_maxent(big, np.tile(r, (n // B, 1)), term.repeat(n // B, 1)),
                 lambda: ops.forward_svf(big, np.tile(p0, (n // B, 1)), term.repeat(n // B, 1),
                                         np.full((n, SIZE * SIZE, 4), 0.25))):
        with pytest.raises(_lib.IrlmxError, match=r"cluster: 1152 workgroups cannot be co-resident \(\d+\)"):
            call()
    torch.cuda.synchronize()


@pytest.mark.parametrize("op", ["backward", "forward"])
def test_exchange_timeout_reruns_bit_identical(world128, monkeypatch, op):
    from irlmx import _lib, ops
    mdp, r, term, p0 = world128
    for o in ("backward", "forward"):
        assert ops.execution_plan(mdp, o)["C"] > 1
    pi = ops.backward_maxent(mdp, r, term)
    if op == "backward":
        run = lambda: ops.backward_maxent(mdp, r, term)
    else:
        run = lambda: ops.forward_svf(mdp, p0, term, pi, max_iter=5000)
    ref = run()
    base = ops.counters()
    monkeypatch.setenv("IRLMX_TEST_DROP_TILE", "1")
    monkeypatch.setenv("IRLMX_TEST_EXCHANGE_TIMEOUT_MS", "50")
    got = run()
    after = ops.counters()
    assert after["rerun_timeout"] == base["rerun_timeout"] + 1
    assert after["sweep_calls"] == base["sweep_calls"] + 1
    for g, e in zip(got if isinstance(got, tuple) else (got,), ref if isinstance(ref, tuple) else (ref,)):
        assert torch.equal(g, e)
    monkeypatch.setenv("IRLMX_STRICT_EXCHANGE", "1")
    with pytest.raises(_lib.IrlmxError, match="halo exchange timed out"):
        run()
    torch.cuda.synchronize()


def test_counters_record_persistent_launches(world):
    from irlmx import ops
    mdp, r, term, p0 = world
    c0 = ops.counters()
    pi = ops.backward_maxent(mdp, r, term)
    ops.forward_svf(mdp, p0, term, pi, max_iter=100)
    c1 = ops.counters()
    assert c1["cluster_launches"] - c0["cluster_launches"] == 2
    assert c1["sweep_calls"] == c0["sweep_calls"] and c1["rerun_not_resident"] == c0["rerun_not_resident"]


def test_numpy_order_rejects_unsorted_ell_rows(dev):
    """The numpy-order entry points sum an ELL row's entries in slot order, which
    is numpy's only for ascending columns (irlmx_dense_to_ell's layout): a model
    whose row slots are reversed is refused with IRLMX_EINVAL and the message,
    the sorted one runs (bit-identical to the oracle's restatement)."""
    import maxent_oracle as O
    from irlmx import DeviceMDP, ops
    size = 5
    S = size * size
    P = O.icy_gridworld_table(size, 0.2)
    good = DeviceMDP.from_dense(P, device=dev, layout="ell")
    r = np.random.default_rng(1).uniform(0.0, 1.0, S)
    tm = ops.terminal_mask([S - 1], S, device=dev)
    pi = ops.backward_maxent_numpy_order(good, np.exp(r), tm)
    assert np.array_equal(pi[0].cpu().numpy(), O.backward_maxent_blas_order(P, [S - 1], r))
    rev = DeviceMDP(good.layout, S, good.n_actions, 1, good.shared, good.row_val.flip(-2).contiguous(),
                    row_idx=good.row_idx.flip(-2).contiguous(), col_idx=good.col_idx, col_val=good.col_val,
                    k_row=good.k_row, k_col=good.k_col, device=dev)
    for call in (lambda: ops.backward_maxent_numpy_order(rev, np.exp(r), tm),
                 lambda: ops.soft_backward(rev, r, O.terminal_reward([S - 1], S), 0.7, numpy_order=True),
                 lambda: ops.value_iteration(rev, r, 0.9, numpy_order=True)):
        with pytest.raises(Exception, match="ascending column order"):
            call()
    # the row order is a table property, computed once per model (irlmx_mdp_properties);
    # with props unknown (0) the entry points check it on the device per call
    from irlmx import _lib
    assert good._struct.props == _lib.PROPS_KNOWN | _lib.PROP_ELL_SORTED
    assert rev._struct.props == _lib.PROPS_KNOWN
    rev._struct.props = 0
    with pytest.raises(Exception, match="ascending column order"):
        ops.backward_maxent_numpy_order(rev, np.exp(r), tm)
    good._struct.props = 0
    assert torch.equal(ops.backward_maxent_numpy_order(good, np.exp(r), tm), pi)


def test_mdp_properties_compact(dev):
    """irlmx_mdp_properties on STENCIL5 tables: IcyGridWorld's collapsed backward
    coefficients have the compact-weight structure, the "stay" variant's (self
    weights inside the grid) do not; at width 256 the backward plan follows the
    property, and with props unknown (0) the per-call device check gives the same
    plan."""
    import ctypes
    from irlmx import DeviceMDP, _lib, ops
    lib = _lib.load()
    for size in (16, 256):
        icy = DeviceMDP.icy_gridworld(size, [0.1, 0.3], device=dev)
        for mdp, compact in ((icy, True), (icy.with_stay(), False)):
            props = ctypes.c_int32(0)
            _lib.check(lib.irlmx_mdp_properties(mdp.struct(), ctypes.byref(props), _lib.stream_ptr(dev)), "props")
            assert props.value == _lib.PROPS_KNOWN | (_lib.PROP_COMPACT if compact else 0), (size, compact)
            if size == 256:
                assert mdp._struct.props == props.value
                plan = ops.execution_plan(mdp, "backward")
                assert (plan["layout"] == 4) == compact, plan
                mdp._struct.props = 0
                assert ops.execution_plan(mdp, "backward") == plan
