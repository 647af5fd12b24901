"""HIP path at the BASELINE configs' full grid sizes (needs an MI355X).

128x128 (configs 3 and 5): the device's backward pass (2*S = 32,768 sweeps on
the cluster plan the planner picks for two instances -- column-strip layout,
R = 4 / G = 14 / C = 32 tiles per instance, halo exchanges, block-boundary
rescaling; the bench's own B = 64 plan is tested in test_gpu_bench_plans.py)
and a forward pass capped at 3,000 sweeps, against the CPU oracle's sparse-operand restatement of the same
reference statements (oracle/maxent_oracle.py ``*_csr``, maxent.py:98-112,
143-159), two instances with distinct slip probabilities.  The reference
itself overflows to NaN beyond 12x12 (its unscaled backward), so the oracle
here is the rescaled restatement, pinned to the reference at small sizes
(tests/test_oracle_golden.py).

256x256 (config 4): size-independent properties of the backward (policy rows
are distributions; instance order does not change any instance's result) --
the CPU restatement would take minutes there.  Layout bit-identity at 256 is
in test_gpu_parity.py::test_width256_quads_bit_identical.
"""

import numpy as np
import pytest

import maxent_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

RTOL = 1e-9       # device vs oracle (float64 both; different summation order only)
CONTRACT = 1e-5   # north-star tolerance


def rel_err(got, ref):
    return float(np.max(np.abs(got - ref)) / np.max(np.abs(ref)))


@pytest.fixture(scope="module")
def dev():
    import __graft_entry__ as g
    g.build()
    import irlmx
    return irlmx.require_device()


def test_config3_grid_vs_sparse_oracle(dev):
    from irlmx import DeviceMDP, ops
    size, slips = 128, (0.1, 0.3)
    n, B = size * size, len(slips)
    rng = np.random.default_rng(128)
    r = rng.uniform(0.0, 1.0, (B, n))
    mdp = DeviceMDP.icy_gridworld(size, list(slips), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    p0 = np.zeros((B, n))
    p0[:, 0] = 1.0
    pi = ops.backward_maxent(mdp, r, tm)
    svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=3000)
    pi_h, svf_h = pi.cpu().numpy(), svf.cpu().numpy()
    for b, slip in enumerate(slips):
        mats = O.icy_gridworld_csr(size, slip)
        pi_ref = O.backward_maxent_csr(mats, [n - 1], r[b])
        e = rel_err(pi_h[b], pi_ref)
        assert e <= CONTRACT and e <= RTOL, (b, "pi", e)
        assert np.argmax(pi_h[b], axis=1).tolist() == np.argmax(pi_ref, axis=1).tolist()
        # forward on the device's own policy: isolates the forward pass
        svf_ref, k_ref = O.forward_svf_csr(mats, p0[b], [n - 1], pi_h[b], max_iter=3000)
        assert int(k[b]) == k_ref == 3000 and int(st[b]) == 2  # capped: IRLMX_MAXITER
        e = rel_err(svf_h[b], svf_ref)
        assert e <= CONTRACT and e <= RTOL, (b, "svf", e)


def test_config4_grid_properties(dev):
    from irlmx import DeviceMDP, ops
    size = 256
    n = size * size
    rng = np.random.default_rng(256)
    slips = [0.1, 0.2, 0.3]
    r = rng.uniform(0.0, 1.0, (3, n))
    tm = ops.terminal_mask([n - 1], n, batch=3, device=dev)
    pi = ops.backward_maxent(DeviceMDP.icy_gridworld(size, slips, device=dev), r, tm).cpu().numpy()
    assert np.all(np.isfinite(pi)) and np.all(pi >= 0.0)
    assert np.max(np.abs(pi.sum(axis=2) - 1.0)) < 1e-12
    # instances are independent: reversing the batch reverses the results, bit for bit
    tm_r = ops.terminal_mask([n - 1], n, batch=3, device=dev)
    pi_r = ops.backward_maxent(DeviceMDP.icy_gridworld(size, slips[::-1], device=dev), r[::-1].copy(), tm_r)
    assert np.array_equal(pi_r.cpu().numpy()[::-1], pi)


@pytest.mark.parametrize("bad", [np.inf, np.nan])
def test_cluster_forward_nonfinite_rerun(dev, bad, monkeypatch):
    """A non-finite start distribution on the cluster shape (64x64, column pairs):
    the block-end check hands the call to the per-sweep shape, whose exact NaN
    bookkeeping stops where the reference's loop does (inf: |inf - inf| = NaN one
    sweep later; NaN: at once).  Asserted: the reference's sweep count (dense
    oracle statements on CSR operands), status NONFINITE, and results bit for bit
    those of the per-sweep shape run directly.  (Values after a NaN stop are not
    compared with the reference: its dense product spreads NaN to every state.)"""
    from irlmx import DeviceMDP, ops
    size = 64
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    tm = ops.terminal_mask([n - 1], n, device=dev)
    r = np.random.default_rng(64).uniform(0.0, 1.0, n)
    pi = ops.backward_maxent(mdp, r, tm)
    p0 = np.zeros(n)
    p0[0] = 0.5
    p0[777] = bad
    svf, k, st = ops.forward_svf(mdp, p0, tm, pi)
    _, k_ref = O.forward_svf_csr(O.icy_gridworld_csr(size, 0.2), p0, [n - 1], pi[0].cpu().numpy())
    assert int(k[0]) == k_ref == (2 if np.isinf(bad) else 1) and int(st[0]) == 1  # IRLMX_NONFINITE
    monkeypatch.setenv("IRLMX_CLUSTER", "0")
    monkeypatch.setenv("IRLMX_FUSED_MAX_STATES", "0")
    svf_s, k_s, st_s = ops.forward_svf(mdp, p0, tm, pi)
    assert torch.equal(svf_s.view(torch.int64), svf.view(torch.int64))  # bit patterns (NaN included)
    assert torch.equal(k_s, k) and torch.equal(st_s, st)


@pytest.mark.parametrize("average", [False, True])
def test_value_iteration_128_vs_sparse_oracle(dev, average):
    """solver.value_iteration / stochastic_value_iteration (solver.py:9-104) at
    128x128 on the device (per-sweep shape) against the sparse-operand oracle:
    identical sweep count, values within 1e-9."""
    from irlmx import DeviceMDP, ops
    size = 128
    n = size * size
    r = np.random.default_rng(17).uniform(0.0, 1.0, n)
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    v, k, st = ops.value_iteration(mdp, r, 0.9, average=average)
    v_ref, k_ref = O.value_iteration_csr(O.icy_gridworld_csr(size, 0.2), r, 0.9, average=average)
    assert int(k[0]) == k_ref and int(st[0]) == 0
    e = rel_err(v[0].cpu().numpy(), v_ref)
    assert e <= CONTRACT and e <= RTOL, e


def test_config2_stay_variant_vs_sparse_oracle(dev):
    """BASELINE config 2's A = 5 variant (IcyGridWorld's four
    moves plus a "stay" action, 64x64, unpinned by the reference's own tests):
    uploaded as a dense [S, S, 5] table (STENCIL5 layout, the stay action on
    the self slot) and checked against the sparse-operand oracle -- backward
    2*S sweeps, a capped and an eps-converged forward (sweep counts equal,
    SVF within 1e-9 relative), soft VI and hard-max VI."""
    import scipy.sparse as sp
    from irlmx import DeviceMDP, _lib, ops
    from irlmx.batch import terminal_reward
    size, n = 64, 64 * 64
    mats = O.icy_gridworld_csr(size, 0.2) + [sp.identity(n, format="csr")]
    dense = np.zeros((n, n, 5))
    for a, m in enumerate(mats):
        c = m.tocoo()
        dense[c.row, c.col, a] = c.data
    mdp = DeviceMDP.from_dense(dense, device=dev)
    del dense
    assert mdp.layout == _lib.LAYOUT_STENCIL5 and mdp.n_actions == 5
    # the bench's construction (bench.py --config c2s): device-built four moves + stay, bit for bit
    built = DeviceMDP.icy_gridworld(size, 0.2, device=dev).with_stay()
    assert built.n_actions == 5 and torch.equal(built.row_val.view(torch.int64), mdp.row_val.view(torch.int64))
    rng = np.random.default_rng(12)
    r = rng.uniform(0.0, 1.0, n)
    term = [n - 1]
    tm = ops.terminal_mask(term, n, device=dev)
    for rb in (r, np.ones(n)):
        pi = ops.backward_maxent(mdp, rb, tm)[0].cpu().numpy()
        ref_pi = O.backward_maxent_csr(mats, term, rb)
        assert np.max(np.abs(pi - ref_pi)) <= 1e-9 * np.max(np.abs(ref_pi))
    p0 = np.zeros(n)
    p0[0] = 1.0
    # (the forward from theta = 1's policy: random rewards mix over millions of sweeps)
    for eps, cap in ((1e-5, 3000), (2e-3, 0)):
        svf, k, st = ops.forward_svf(mdp, p0, tm, ref_pi, eps=eps, max_iter=cap)
        ref_svf, ref_k = O.forward_svf_csr(mats, p0, term, ref_pi, eps=eps, max_iter=cap or None)
        assert int(k[0]) == ref_k, (eps, cap, int(k[0]), ref_k)
        assert np.max(np.abs(svf[0].cpu().numpy() - ref_svf)) <= 1e-9 * np.max(np.abs(ref_svf))
    v, kv, _ = ops.value_iteration(mdp, r, 0.9)
    ref_v, ref_kv = O.value_iteration_csr(mats, r, 0.9)
    assert int(kv[0]) == ref_kv
    assert np.max(np.abs(v[0].cpu().numpy() - ref_v)) <= 1e-12 * np.max(np.abs(ref_v))
    cpi, cv, ks, _ = ops.soft_backward(mdp, r, terminal_reward(term, n, 1, dev), 0.7)
    ref_cpi, ref_cv, ref_ks = O.soft_backward_csr(mats, term, r, 0.7)
    assert int(ks[0]) == ref_ks
    assert np.max(np.abs(cpi[0].cpu().numpy() - ref_cpi)) <= 1e-9 * np.max(np.abs(ref_cpi))
    assert np.max(np.abs(cv[0].cpu().numpy() - ref_cv)) <= 1e-9 * np.max(np.abs(ref_cv))


def ell_model(mats, dev):
    """A DeviceMDP in the ELL layout built on the host from per-action CSR
    matrices (the layout irlmx_dense_to_ell produces: targets / sources of each
    state ascending, unused slots pointing at the state itself with value 0)."""
    import scipy.sparse as sp
    from irlmx import DeviceMDP, _lib
    n, A = mats[0].shape[0], len(mats)
    union = sum(abs(m) for m in mats).tocsr()
    union.sort_indices()

    def form(u, ms):
        cnt = np.diff(u.indptr)
        k = max(1, int(cnt.max()))
        rows = np.repeat(np.arange(n), cnt)
        slot = np.arange(u.indices.size) - np.repeat(u.indptr[:-1], cnt)
        idx = np.tile(np.arange(n), (k, 1))
        idx[slot, rows] = u.indices
        val = np.zeros((A, k, n))
        for a, m in enumerate(ms):
            val[a, slot, rows] = np.asarray(m[rows, u.indices]).reshape(-1)
        return k, idx, val

    k_row, ri, rv = form(union, mats)
    ut = union.T.tocsr()
    ut.sort_indices()
    k_col, ci, cv = form(ut, [m.T.tocsr() for m in mats])
    t = lambda x, dt: torch.as_tensor(x[None], dtype=dt, device=dev).contiguous()
    return DeviceMDP(_lib.LAYOUT_ELL, n, A, 1, True, t(rv, torch.float64), row_idx=t(ri, torch.int32),
                     col_idx=t(ci, torch.int32), col_val=t(cv, torch.float64), k_row=k_row, k_col=k_col, device=dev)


def test_ell_grid_shape_at_128(dev, monkeypatch):
    """A 128x128 IcyGridWorld in the generic ELL layout (S = 16384 > one CU):
    backward, forward, soft VI and VI run on the persistent grid shape, bit for
    bit equal to the per-sweep shape (also the unscaled, overflowing backward),
    and the backward and capped forward within 1e-9 of the CSR oracle."""
    from irlmx import ops
    from irlmx.batch import terminal_reward
    size, n = 128, 128 * 128
    mats = O.icy_gridworld_csr(size, 0.2)
    mdp = ell_model(mats, dev).with_batch(2)
    assert mdp.k_row <= 5 and mdp.k_col <= 5
    for op in ("backward", "forward", "soft_backward", "value_iteration"):
        assert ops.execution_plan(mdp, op)["shape"] == "grid", op
    rng = np.random.default_rng(99)
    r = rng.uniform(0.0, 1.0, (2, n))
    tm = ops.terminal_mask([n - 1], n, batch=2, device=dev)
    p0 = np.zeros((2, n))
    p0[:, 0] = 1.0
    phi = terminal_reward([n - 1], n, 2, dev)

    def run():
        pi = ops.backward_maxent(mdp, r, tm)
        # (a converged forward on the unit-reward policy: random rewards mix over millions of sweeps)
        pi1 = ops.backward_maxent(mdp, np.ones((2, n)), tm)
        return (pi, ops.forward_svf(mdp, p0, tm, pi, max_iter=3000), ops.forward_svf(mdp, p0, tm, pi1, eps=1e-2),
                ops.soft_backward(mdp, r, phi, 0.7), ops.value_iteration(mdp, r, 0.9),
                ops.backward_maxent(mdp, r, tm, rescale=False))

    got = run()
    monkeypatch.setenv("IRLMX_GRID", "0")
    assert ops.execution_plan(mdp, "forward")["shape"] == "sweep"
    ref = run()

    def bits(x):
        return x.view(torch.int64) if x.dtype == torch.float64 else x

    flat = lambda t: list(t) if isinstance(t, tuple) else [t]
    for g_, r_ in zip(got, ref):
        for x, y in zip(flat(g_), flat(r_)):
            assert torch.equal(bits(x), bits(y))
    assert bool(torch.isnan(got[5]).all())                  # the reference's overflow: NaN everywhere
    pi = got[0][0].cpu().numpy()
    pi_ref = O.backward_maxent_csr(mats, [n - 1], r[0])
    assert rel_err(pi, pi_ref) <= RTOL
    svf_ref, k_ref = O.forward_svf_csr(mats, p0[0], [n - 1], pi, max_iter=3000)
    assert int(got[1][1][0]) == k_ref == 3000 and rel_err(got[1][0][0].cpu().numpy(), svf_ref) <= RTOL


def random_sparse_mats(n, A, n_succ, seed, n_offsets=32):
    """Per-action CSR matrices of a random sparse MDP: state s reaches n_succ
    distinct targets (s + o) mod n, o drawn per state from one fixed set of
    n_offsets random offsets (so no state has more than n_offsets sources), each
    action a random distribution over a random subset of them."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    offsets = rng.choice(np.arange(1, n), n_offsets, replace=False)
    pick = np.argsort(rng.random((n, n_offsets)), axis=1)[:, :n_succ]
    tgt = np.sort((np.arange(n)[:, None] + offsets[pick]) % n, axis=1)
    mats = []
    for _ in range(A):
        w = rng.random((n, n_succ)) * (rng.random((n, n_succ)) < 0.5)
        w[np.arange(n), rng.integers(0, n_succ, n)] += 0.5  # at least one target per action
        w /= w.sum(axis=1, keepdims=True)
        mats.append(sp.csr_matrix((w.ravel(), tgt.ravel(), np.arange(0, n * n_succ + 1, n_succ)), shape=(n, n)))
    return mats


@pytest.mark.parametrize("n_succ,kmax", [(12, 16), (24, 32)])
def test_ell_grid_shape_wide_rows(dev, monkeypatch, n_succ, kmax):
    """Generic sparse models with 9-32 slots per state (S = 6000 > one CU): the
    linear loops (backward, forward) on the persistent grid shape with 16 / 32
    slots per state in registers, soft VI and VI there too up to 16 slots -- bit
    for bit the per-sweep shape (IRLMX_GRID=0), and the backward and capped
    forward within 1e-9 of the CSR oracle."""
    from irlmx import ops
    from irlmx.batch import terminal_reward
    n, B = 6000, 2
    mats = random_sparse_mats(n, 4, n_succ, seed=n_succ)
    mdp = ell_model(mats, dev).with_batch(B)
    assert 8 < mdp.k_row <= kmax and mdp.k_col <= 32, (mdp.k_row, mdp.k_col)
    for op in ("backward", "forward"):
        assert ops.execution_plan(mdp, op)["shape"] == "grid", op
    for op in ("soft_backward", "value_iteration"):
        assert ops.execution_plan(mdp, op)["shape"] == ("grid" if kmax == 16 else "sweep"), op
    rng = np.random.default_rng(n_succ)
    r = rng.uniform(0.0, 1.0, (B, n))
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    p0 = np.zeros((B, n))
    p0[:, 0] = 1.0
    phi = terminal_reward([n - 1], n, B, dev)

    def run():
        pi = ops.backward_maxent(mdp, r, tm)
        return (pi, ops.forward_svf(mdp, p0, tm, pi, max_iter=500), ops.soft_backward(mdp, r, phi, 0.7),
                ops.value_iteration(mdp, r, 0.9))

    got = run()
    monkeypatch.setenv("IRLMX_GRID", "0")
    assert ops.execution_plan(mdp, "forward")["shape"] == "sweep"
    ref = run()
    monkeypatch.delenv("IRLMX_GRID")

    def bits(x):
        return x.view(torch.int64) if x.dtype == torch.float64 else x

    flat = lambda t: list(t) if isinstance(t, tuple) else [t]
    for g_, r_ in zip(got, ref):
        for x, y in zip(flat(g_), flat(r_)):
            assert torch.equal(bits(x), bits(y))
    pi = got[0][1].cpu().numpy()
    assert rel_err(pi, O.backward_maxent_csr(mats, [n - 1], r[1])) <= RTOL
    svf_ref, k_ref = O.forward_svf_csr(mats, p0[1], [n - 1], pi, max_iter=500)
    assert int(got[1][1][1]) == k_ref and rel_err(got[1][0][1].cpu().numpy(), svf_ref) <= RTOL
