"""Persistent dense shape (IRLMX_SHAPE_DENSE_GRID, csrc/dense_grid.hip).

The forward (maxent.py:98-112), the collapsed backward (maxent.py:143-159) and
soft VI / VI (maxent.py:326-341, solver.py:40-50 / 95-100) of DENSE models in
one launch per call, each workgroup holding its rows of the S x S matrices in
registers and the swept vector exchanged as tagged granules.
Checked against the per-sweep dense kernels (IRLMX_DENSE_GRID=0: one launch per
sweep, csrc/dense.hip) and the dense oracle: sweep counts and statuses
identical, values within 1e-12 relative (only the summation order of each row
dot differs); the loop rules at their edges (max_iter cap, non-finite policy,
non-finite partition values, rescale off); every (rows per workgroup, columns
per thread) instantiation the planner can pick; the per-sweep rerun when the
workgroups cannot all run at once.
"""

import numpy as np
import pytest

import maxent_oracle as O
from conftest import load_golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

RTOL = 1e-12


@pytest.fixture(scope="module")
def dev():
    import __graft_entry__ as g
    g.build()
    import irlmx
    return irlmx.require_device()


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    assert np.array_equal(np.isnan(a), np.isnan(b))
    fin = np.isfinite(b)
    return float(np.max(np.abs(a[fin] - b[fin])) / max(np.max(np.abs(b[fin])), 1e-300)) if fin.any() else 0.0


def dense_model(dev, n, A, batch, shared, seed):
    """A DENSE-layout model: one random table for all instances (shared) or one per instance."""
    from irlmx import DeviceMDP, _lib
    if shared:
        P, _, _, _ = O.random_dense_mdp(n, A, seed=seed)
        return DeviceMDP.from_dense(P, device=dev, layout="dense").with_batch(batch), [P] * batch
    Ps = [O.random_dense_mdp(n, A, seed=seed + b)[0] for b in range(batch)]
    parts = [DeviceMDP.from_dense(P, device=dev, layout="dense") for P in Ps]
    mdp = DeviceMDP(_lib.LAYOUT_DENSE, n, A, batch, False, torch.cat([p.row_val for p in parts]),
                    col_val=torch.cat([p.col_val for p in parts]), k_row=n, k_col=n, device=dev)
    return mdp, Ps


def both_shapes(monkeypatch, fn):
    """fn() on the dense grid shape, then on the per-sweep dense shape."""
    monkeypatch.delenv("IRLMX_DENSE_GRID", raising=False)
    grid = fn()
    monkeypatch.setenv("IRLMX_DENSE_GRID", "0")
    sweep = fn()
    monkeypatch.delenv("IRLMX_DENSE_GRID", raising=False)
    return grid, sweep


CASES = [  # S, A, B, shared
    (7, 3, 1, True), (64, 4, 2, False), (300, 4, 5, True), (513, 3, 3, False), (1037, 4, 2, True),
    (2048, 4, 1, True), (2048, 4, 2, False),
]


@pytest.mark.parametrize("n,A,batch,shared", CASES)
def test_dense_grid_vs_per_sweep(dev, monkeypatch, n, A, batch, shared):
    from irlmx import ops
    mdp, _ = dense_model(dev, n, A, batch, shared, seed=n)
    for op in ("forward", "backward"):
        plan = ops.execution_plan(mdp, op)
        assert plan["shape"] == "dense-grid", (op, plan)
        assert plan["R"] * plan["C"] >= n and plan["spt"] * 512 >= n and plan["C"] * batch <= 256, plan
    rng = np.random.default_rng(n + batch)
    r = rng.uniform(0.0, 1.0, (batch, n))
    tm = ops.terminal_mask([n - 1], n, batch=batch, device=dev)
    p0 = np.zeros((batch, n))
    p0[:, 0] = 1.0

    def run():
        pi = ops.backward_maxent(mdp, r, tm)
        svf, k, st = ops.forward_svf(mdp, p0, tm, pi)
        return pi.cpu().numpy(), svf.cpu().numpy(), k.cpu().numpy(), st.cpu().numpy()

    (pi_g, svf_g, k_g, st_g), (pi_s, svf_s, k_s, st_s) = both_shapes(monkeypatch, run)
    assert rel(pi_g, pi_s) <= RTOL
    assert np.array_equal(k_g, k_s) and np.array_equal(st_g, st_s), (k_g, k_s)
    assert np.all(st_g == 0)
    # forward on the SAME policy (isolates the forward pass from the backward's rounding)
    monkeypatch.setenv("IRLMX_DENSE_GRID", "0")
    svf_s2, k_s2, _ = ops.forward_svf(mdp, p0, tm, pi_g)
    monkeypatch.delenv("IRLMX_DENSE_GRID")
    assert np.array_equal(k_g, k_s2.cpu().numpy())
    assert rel(svf_g, svf_s2.cpu().numpy()) <= 1e-11


def test_dense_grid_vs_oracle_2048(dev):
    """The seeded S = 2048 dense MDP (tests/golden/dense2048.npz, the dense oracle's
    outputs): backward and forward on the dense grid shape (16 rows x 4 columns per
    thread, 128 workgroups), sweep count identical, 1e-9."""
    from irlmx import DeviceMDP, ops
    z = load_golden("dense2048")
    P, r, term, p0 = O.random_dense_mdp()
    mdp = DeviceMDP.from_dense(P, device=dev)
    plan = ops.execution_plan(mdp, "backward")
    assert (plan["shape"], plan["R"], plan["spt"], plan["C"], plan["G"]) == ("dense-grid", 16, 4, 128, 0)
    tm = ops.terminal_mask(term, 2048, device=dev)
    pi = ops.backward_maxent(mdp, r, tm)[0].cpu().numpy()
    assert rel(pi, z["pi"]) <= 1e-9
    svf, k, st = ops.forward_svf(mdp, p0, tm, pi)
    assert int(k[0]) == int(z["k_f"]) and int(st[0]) == 0
    assert rel(svf[0].cpu().numpy(), z["svf"]) <= 1e-9


@pytest.mark.parametrize("n,rb,xcd", [(200, 4, 0), (200, 8, 0), (200, 16, 0), (200, 32, 0), (200, 64, 0),
                                      (200, 16, 1), (700, 4, 0), (700, 8, 0), (700, 16, 0), (700, 32, 0),
                                      (700, 32, 1), (1500, 8, 0), (1500, 16, 0)])
def test_dense_grid_every_instantiation(dev, monkeypatch, n, rb, xcd):
    """IRLMX_DENSE_GRID_RB forces each (rows per workgroup, columns per thread)
    pair the planner can pick (S = 200 / 700 / 1500: 1, 2, 4 columns per thread;
    ragged last workgroup), IRLMX_DENSE_GRID_XCD=1 one instance's workgroups onto
    one XCD (plain stores): backward and a 400-sweep forward against the per-sweep
    dense shape, and against the dense oracle up to S = 700."""
    monkeypatch.setenv("IRLMX_DENSE_GRID_XCD", str(xcd))
    from irlmx import ops
    mdp, (P,) = dense_model(dev, n, 3, 1, True, seed=7 * n)
    r = np.random.default_rng(rb).uniform(0.0, 1.0, n)
    tm = ops.terminal_mask([n - 1], n, device=dev)
    p0 = np.zeros(n)
    p0[0] = 1.0

    def run():
        pi = ops.backward_maxent(mdp, r, tm)[0].cpu().numpy()
        svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=400)
        return pi, svf[0].cpu().numpy(), int(k[0]), int(st[0])

    monkeypatch.setenv("IRLMX_DENSE_GRID_RB", str(rb))
    plan = ops.execution_plan(mdp, "backward")
    assert plan["shape"] == "dense-grid" and plan["R"] == rb and plan["G"] == xcd, plan
    assert ops.execution_plan(mdp, "forward")["R"] == rb
    (pi, svf, k, st), (pi_s, svf_s, k_s, st_s) = both_shapes(monkeypatch, run)
    monkeypatch.delenv("IRLMX_DENSE_GRID_RB")
    monkeypatch.delenv("IRLMX_DENSE_GRID_XCD")
    assert rel(pi, pi_s) <= RTOL and (k, st) == (k_s, st_s)
    assert rel(svf, svf_s) <= 1e-11
    if n <= 700:
        assert rel(pi, O.backward_maxent(P, [n - 1], r, rescale=True)) <= 1e-9
        svf_ref, k_ref = O.forward_svf(P, p0, [n - 1], pi, max_iter=400)
        assert k == k_ref and st == (0 if k_ref < 400 else 2)
        assert rel(svf, svf_ref) <= 1e-9


@pytest.mark.parametrize("n,batch,plan", [(256, 1, (8, 32, 1)), (512, 2, (16, 32, 1)), (1024, 1, (32, 32, 1)),
                                          (1024, 8, (32, 32, 1)), (512, 8, (16, 32, 1)), (2048, 1, (16, 128, 0)), (2048, 2, (16, 128, 0))])
def test_dense_grid_planner(dev, n, batch, plan):
    """The planner's measured preference: one XCD per instance
    group at the fewest rows per workgroup that fit, else >= 8 rows and at most
    128 workgroups per instance spread over the chip; (rows, workgroups per
    instance, XCD-grouped)."""
    from irlmx import ops
    mdp, _ = dense_model(dev, n, 2, batch, True, seed=1)
    for op in ("forward", "backward"):
        p = ops.execution_plan(mdp, op)
        assert (p["shape"], p["R"], p["C"], p["G"]) == ("dense-grid",) + plan, (op, p)


@pytest.mark.parametrize("n,A,batch,plan", [(256, 4, 1, (8, 32, 1, 4)), (512, 4, 1, (4, 128, 0, 4)),
                                            (1024, 4, 1, (4, 256, 0, 4)), (256, 6, 2, (8, 32, 1, 8))])
def test_dense_bellman_grid_planner(dev, n, A, batch, plan):
    """Soft VI / VI plans: one XCD per instance group only at <= 8
    states per workgroup, else the fewest states per workgroup spread over the
    chip; (states per workgroup, workgroups per instance, XCD-grouped, actions
    compiled)."""
    from irlmx import ops
    mdp, _ = dense_model(dev, n, A, batch, True, seed=2)
    for op in ("soft_backward", "value_iteration"):
        p = ops.execution_plan(mdp, op)
        assert (p["shape"], p["R"], p["C"], p["G"], p["layout"]) == ("dense-grid",) + plan, (op, p)


def test_dense_grid_loop_edges(dev, monkeypatch):
    """The loop rules at their edges, dense grid vs per-sweep dense shape: a
    max_iter cap (status MAXITER, values after exactly 5 sweeps), a non-finite
    policy entry (svf NaN, 1 sweep, NONFINITE: the reference's dense product),
    a NaN reward (every partition value NaN: bwd_nonfinite_rule), and rescale off
    with a reward large enough to overflow (inf partition values)."""
    from irlmx import ops
    n, B = 300, 3
    mdp, _ = dense_model(dev, n, 4, B, True, seed=3)
    rng = np.random.default_rng(5)
    r = rng.uniform(0.0, 1.0, (B, n))
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    p0 = np.zeros((B, n))
    p0[:, 0] = 1.0
    pi = ops.backward_maxent(mdp, r, tm).cpu().numpy()
    pi[1, 17, 2] = np.nan  # instance 1: non-finite policy

    def fwd(**kw):
        svf, k, st = ops.forward_svf(mdp, p0, tm, pi, **kw)
        return svf.cpu().numpy(), k.cpu().numpy(), st.cpu().numpy()

    for kw in ({}, {"max_iter": 5}):
        (s_g, k_g, st_g), (s_s, k_s, st_s) = both_shapes(monkeypatch, lambda: fwd(**kw))
        assert np.array_equal(k_g, k_s) and np.array_equal(st_g, st_s), (kw, k_g, k_s, st_g, st_s)
        assert int(k_g[1]) == 1 and int(st_g[1]) == 1 and np.all(np.isnan(s_g[1]))
        if kw:
            assert list(k_g) == [5, 1, 5] and list(st_g) == [2, 1, 2]
        assert rel(s_g, s_s) <= 1e-11
    r_bad = r.copy()
    r_bad[2, 9] = np.nan  # instance 2: NaN partition values from the first sweep on
    assert ops.execution_plan(mdp, "backward")["shape"] == "dense-grid"
    g, s = both_shapes(monkeypatch, lambda: ops.backward_maxent(mdp, r_bad, tm).cpu().numpy())
    assert np.all(np.isnan(g[2])) and not np.any(np.isnan(g[:2]))
    assert np.array_equal(np.isnan(g), np.isnan(s)) and rel(g, s) <= RTOL
    # rescale off: 2S = 120 unscaled sweeps stay finite at r < 1 (row sums A = 4: growth
    # <= 4e per sweep), and overflow to inf (then NaN) at r = 40 (instance 0)
    n2 = 60
    mdp2, P2 = dense_model(dev, n2, 4, B, True, seed=4)
    r2 = rng.uniform(0.0, 1.0, (B, n2))
    r2[0] = 40.0
    tm2 = ops.terminal_mask([n2 - 1], n2, batch=B, device=dev)
    assert ops.execution_plan(mdp2, "backward", rescale=False)["shape"] == "dense-grid"
    g, s = both_shapes(monkeypatch, lambda: ops.backward_maxent(mdp2, r2, tm2, rescale=False).cpu().numpy())
    assert np.all(np.isnan(g[0])) and not np.any(np.isnan(g[1:]))
    assert np.array_equal(np.isnan(g), np.isnan(s)) and rel(g, s) <= RTOL
    assert rel(g[1], O.backward_maxent(P2[1], [n2 - 1], r2[1], rescale=False)) <= 1e-9


def test_dense_grid_not_resident_rerun(dev, monkeypatch):
    """A launch whose workgroups cannot all run at once (IRLMX_TEST_NOT_RESIDENT:
    the rendezvous waits for one workgroup more than launched) reruns the call on
    the per-sweep dense shape, with its results, and counts the rerun (backward
    and soft VI)."""
    from irlmx import ops
    n = 400
    mdp, _ = dense_model(dev, n, 4, 2, True, seed=11)
    r = np.random.default_rng(1).uniform(0.0, 1.0, (2, n))
    tm = ops.terminal_mask([n - 1], n, batch=2, device=dev)
    monkeypatch.setenv("IRLMX_DENSE_GRID", "0")
    ref = ops.backward_maxent(mdp, r, tm)
    monkeypatch.delenv("IRLMX_DENSE_GRID")
    before = ops.counters()
    monkeypatch.setenv("IRLMX_TEST_NOT_RESIDENT", "1")
    got = ops.backward_maxent(mdp, r, tm)
    monkeypatch.delenv("IRLMX_TEST_NOT_RESIDENT")
    after = ops.counters()
    assert after["rerun_not_resident"] == before["rerun_not_resident"] + 1
    assert after["sweep_calls"] == before["sweep_calls"] + 1   # the per-sweep rerun is counted
    assert torch.equal(got, ref)
    # soft VI likewise
    from irlmx.batch import terminal_reward
    phi = terminal_reward([n - 1], n, 2, dev)
    monkeypatch.setenv("IRLMX_DENSE_GRID", "0")
    ref = ops.soft_backward(mdp, r, phi, 0.7)
    monkeypatch.delenv("IRLMX_DENSE_GRID")
    assert ops.execution_plan(mdp, "soft_backward")["shape"] == "dense-grid"
    before = ops.counters()
    monkeypatch.setenv("IRLMX_TEST_NOT_RESIDENT", "1")
    got = ops.soft_backward(mdp, r, phi, 0.7)
    monkeypatch.delenv("IRLMX_TEST_NOT_RESIDENT")
    after = ops.counters()
    assert after["rerun_not_resident"] == before["rerun_not_resident"] + 1
    assert after["sweep_calls"] == before["sweep_calls"] + 1
    for x, y in zip(got, ref):
        assert torch.equal(x, y)


def test_dense_grid_exchange_timeout_rerun(dev, monkeypatch):
    """One workgroup of a dense-grid launch leaves right after the rendezvous
    (IRLMX_TEST_DROP_TILE) and the others' all-gather times out
    (IRLMX_TEST_EXCHANGE_TIMEOUT_MS): the forward, the backward and soft VI
    rerun on the per-sweep dense shape with its results, counted as
    rerun_timeout and sweep_calls; IRLMX_STRICT_EXCHANGE=1 reports it instead."""
    from irlmx import _lib, ops
    from irlmx.batch import terminal_reward
    n = 400
    mdp, _ = dense_model(dev, n, 4, 2, True, seed=11)
    r = np.random.default_rng(1).uniform(0.0, 1.0, (2, n))
    tm = ops.terminal_mask([n - 1], n, batch=2, device=dev)
    phi = terminal_reward([n - 1], n, 2, dev)
    p0 = np.zeros((2, n))
    p0[:, 0] = 1.0
    pi = ops.backward_maxent(mdp, r, tm)
    calls = {"backward": lambda: ops.backward_maxent(mdp, r, tm),
             "forward": lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=500),
             "soft_backward": lambda: ops.soft_backward(mdp, r, phi, 0.7)}
    for op, run in calls.items():
        assert ops.execution_plan(mdp, op)["shape"] == "dense-grid", op
        monkeypatch.setenv("IRLMX_DENSE_GRID", "0")
        ref = run()
        monkeypatch.delenv("IRLMX_DENSE_GRID")
        before = ops.counters()
        monkeypatch.setenv("IRLMX_TEST_DROP_TILE", "1")
        monkeypatch.setenv("IRLMX_TEST_EXCHANGE_TIMEOUT_MS", "50")
        got = run()
        after = ops.counters()
        assert after["rerun_timeout"] == before["rerun_timeout"] + 1, op
        assert after["sweep_calls"] == before["sweep_calls"] + 1, op
        for x, y in zip(got if isinstance(got, tuple) else (got,), ref if isinstance(ref, tuple) else (ref,)):
            assert torch.equal(x, y), op
        monkeypatch.setenv("IRLMX_STRICT_EXCHANGE", "1")
        with pytest.raises(_lib.IrlmxError, match="dense grid shape: exchange timed out"):
            run()
        for k in ("IRLMX_TEST_DROP_TILE", "IRLMX_TEST_EXCHANGE_TIMEOUT_MS", "IRLMX_STRICT_EXCHANGE"):
            monkeypatch.delenv(k)
    torch.cuda.synchronize()


BELLMAN_CASES = [  # S, A, B, shared
    (7, 3, 1, True), (64, 4, 2, False), (300, 4, 3, True), (513, 4, 2, True), (1000, 4, 1, True),
    (200, 5, 2, True), (700, 6, 1, True), (130, 8, 3, False),
]


@pytest.mark.parametrize("n,A,batch,shared", BELLMAN_CASES)
def test_dense_grid_soft_vi_and_vi(dev, monkeypatch, n, A, batch, shared):
    """Soft VI (discount 0.7; pi and value) and VI (max and mean over actions) on
    the dense grid shape against the per-sweep dense kernels: sweep counts and
    statuses identical, values and policies within 1e-12; and against the dense
    oracle for the first instance."""
    from irlmx import ops
    from irlmx.batch import terminal_reward
    mdp, Ps = dense_model(dev, n, A, batch, shared, seed=3 * n + A)
    for op in ("soft_backward", "value_iteration"):
        plan = ops.execution_plan(mdp, op)
        assert plan["shape"] == "dense-grid" and plan["layout"] == (4 if A <= 4 else 8), (op, plan)
    r = np.random.default_rng(n).uniform(0.0, 1.0, (batch, n))
    phi = terminal_reward([n - 1], n, batch, dev)

    def run():
        pi, v, k, st = ops.soft_backward(mdp, r, phi, 0.7)
        vi, kv, stv = ops.value_iteration(mdp, r, 0.9)
        va, kva, sta = ops.value_iteration(mdp, r, 0.9, average=True)
        return [x.cpu().numpy() for x in (pi, v, k, st, vi, kv, stv, va, kva, sta)]

    g, sw = both_shapes(monkeypatch, run)
    for i in (2, 3, 5, 6, 8, 9):  # sweep counts and statuses
        assert np.array_equal(g[i], sw[i]), (i, g[i], sw[i])
    for i in (0, 1, 4, 7):
        assert rel(g[i], sw[i]) <= RTOL, i
    pi_ref, v_ref, k_ref = O.soft_backward(Ps[0], [n - 1], r[0], 0.7)
    assert int(g[2][0]) == k_ref
    assert rel(g[0][0], pi_ref) <= 1e-9 and rel(g[1][0], v_ref) <= 1e-9
    vv_ref, kv_ref = O.value_iteration(Ps[0], r[0], 0.9)
    assert int(g[5][0]) == kv_ref and rel(g[4][0], vv_ref) <= 1e-9


@pytest.mark.parametrize("n,A,rb", [(300, 4, 4), (300, 4, 8), (300, 4, 16), (900, 4, 4), (900, 4, 8),
                                    (200, 7, 2), (200, 7, 4), (200, 7, 8), (800, 7, 4)])
def test_dense_bellman_grid_every_instantiation(dev, monkeypatch, n, A, rb):
    """Every (actions compiled, rows, columns per thread) instantiation of the
    Bellman kernel, forced by IRLMX_DENSE_GRID_RB (spread over the chip), with a
    sweep cap: soft VI and VI against the per-sweep dense kernels."""
    from irlmx import ops
    from irlmx.batch import terminal_reward
    mdp, _ = dense_model(dev, n, A, 1, True, seed=n + rb)
    monkeypatch.setenv("IRLMX_DENSE_GRID_RB", str(rb))
    monkeypatch.setenv("IRLMX_DENSE_GRID_XCD", "0")
    plan = ops.execution_plan(mdp, "soft_backward")
    assert plan["shape"] == "dense-grid" and plan["R"] == rb and plan["G"] == 0, plan
    r = np.random.default_rng(rb).uniform(0.0, 1.0, (1, n))
    phi = terminal_reward([n - 1], n, 1, dev)

    def run():
        pi, v, k, st = ops.soft_backward(mdp, r, phi, 0.7, max_iter=40)
        vi, kv, stv = ops.value_iteration(mdp, r, 0.9)
        return [x.cpu().numpy() for x in (pi, v, k, st, vi, kv, stv)]

    g, sw = both_shapes(monkeypatch, run)
    assert int(g[2][0]) == int(sw[2][0]) and int(g[3][0]) == int(sw[3][0])
    assert np.array_equal(g[5], sw[5]) and np.array_equal(g[6], sw[6])
    for i in (0, 1, 4):
        assert rel(g[i], sw[i]) <= RTOL, i
