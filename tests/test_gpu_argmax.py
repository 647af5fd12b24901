"""Argmax / policy indices end to end, device only (needs an MI355X).

North star: "bit-exact on indices/argmax".  These tests never feed the device
a reference value vector: every index below comes from a chain that runs on
the device from the reward, compared with the reference's own output
(tests/golden, made by importing the reference, tools/gen_golden.py).

* Greedy policy (solver.py:107-152): device value_iteration -> device
  optimal_policy_from_value, and the drop-in solver.optimal_policy(world, ...),
  against the reference's ``opt_policy`` -- np.array_equal, ties (first index)
  included (det4 has nine states with two exactly tied successors).
* Argmax of the backward policy (maxent.py:159, 341) at every reference-pinned
  case, ties included (see test_backward_policy_argmax for how ties are
  reproduced).
"""

import numpy as np
import pytest

import maxent_oracle as O
from conftest import load_golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    import __graft_entry__ as g
    g.build()
    import irlmx
    return irlmx.require_device()


class GridWorldStandIn:
    """The reference GridWorld API solver.optimal_policy uses (gridworld.py:14-122):
    size, actions, n_states / n_actions, state_index_transition, p_transition."""

    def __init__(self, size, p_transition):
        self.size = size
        self.n_states, self.n_actions = size * size, 4
        self.actions = O.ACTIONS
        self.p_transition = p_transition

    def state_index_transition(self, s, a):
        return O.intended_successor(self.size, s, a)


def _argmax_report(got, ref):
    bad = np.flatnonzero(got != ref)
    return f"{bad.size} states differ: " + ", ".join(f"s={s} got {got[s]} ref {ref[s]}" for s in bad[:8])


def test_value_iteration_policy_chain(dev):
    """solver.optimal_policy (solver.py:127-152) = value_iteration on the device,
    then the greedy successor argmax on the device, for every golden VI case with
    a greedy policy (5x5 and 16x16, discount 0.7 / 0.9) and det4 (deterministic
    4x4 GridWorld, discount 0.5, nine states with exact two-way ties)."""
    import solver as S
    from irlmx import DeviceMDP, ops
    z = load_golden("vi")
    cases = [str(c) for c in z["names"] if str(c) + "__opt_policy" in z]
    assert len(cases) == 4
    for c in cases:
        size = int(z[c + "__size"])
        mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
        v, k, _ = ops.value_iteration(mdp, z[c + "__reward"], float(z[c + "__discount"]))
        assert int(k[0]) == int(z[c + "__k"]), c
        succ = torch.as_tensor(S.successor_table(GridWorldStandIn(size, None)), device=dev)
        pol = ops.optimal_policy(succ, v[0]).cpu().numpy()[0]
        assert np.array_equal(pol, z[c + "__opt_policy"]), (c, _argmax_report(pol, z[c + "__opt_policy"]))
        # the drop-in path: numpy table in, numpy indices out
        world = GridWorldStandIn(size, O.icy_gridworld_table(size, 0.2))
        pol2 = S.optimal_policy(world, z[c + "__reward"], float(z[c + "__discount"]))
        assert np.array_equal(pol2, z[c + "__opt_policy"]), (c, _argmax_report(pol2, z[c + "__opt_policy"]))
    world = GridWorldStandIn(4, O.gridworld_table(4))
    mdp = DeviceMDP.gridworld(4, device=dev)
    v, k, _ = ops.value_iteration(mdp, z["det4__reward"], 0.5)
    assert int(k[0]) == int(z["det4__k"])
    assert np.array_equal(v[0].cpu().numpy(), z["det4__value"])   # deterministic moves: exact arithmetic
    succ = torch.as_tensor(S.successor_table(world), device=dev)
    pol = ops.optimal_policy(succ, v[0]).cpu().numpy()[0]
    assert np.array_equal(pol, z["det4__opt_policy"]), _argmax_report(pol, z["det4__opt_policy"])
    pol2 = S.optimal_policy(world, z["det4__reward"], 0.5)
    assert np.array_equal(pol2, z["det4__opt_policy"]), _argmax_report(pol2, z["det4__opt_policy"])


def test_config1_policy_chain(dev):
    """BASELINE config 1 (src/main.py): the expert's greedy policy from the
    device's own value iteration equals the reference's."""
    import solver as S
    z = load_golden("config1")
    world = GridWorldStandIn(5, z["p_transition"])
    pol = S.optimal_policy(world, z["reward"], 0.7)
    assert np.array_equal(pol, z["opt_policy"]), _argmax_report(pol, z["opt_policy"])


def _pinned_backward_cases():
    """(name, p_transition, terminal, reward, reference pi) of every reference-pinned
    backward-policy case with a finite reference policy: maxent_small (5x5 - 12x12),
    config 1's pi1 (maxent.py:159)."""
    z = load_golden("maxent_small")
    for c in [str(n) for n in z["names"]]:
        if not np.isfinite(z[c + "__pi"]).all():
            continue
        P = O.icy_gridworld_table(int(z[c + "__size"]), float(z[c + "__p_slip"]))
        yield c, P, [int(t) for t in z[c + "__terminal"]], z[c + "__reward"], z[c + "__pi"]
    z = load_golden("config1")
    yield "config1_pi1", z["p_transition"], [int(t) for t in z["terminal"]], np.ones(25), z["pi1"]


def _pinned_causal_cases():
    z = load_golden("causal_small")
    for c in [str(n) for n in z["names"]]:
        size = int(z[c + "__size"])
        yield (c, O.icy_gridworld_table(size, 0.2), [int(t) for t in z[c + "__terminal"]], z[c + "__reward"],
               float(z[c + "__discount"]), z[c + "__pi"])
    z = load_golden("config1")
    yield "config1_cpi1", z["p_transition"], [int(t) for t in z["terminal"]], np.ones(25), 0.7, z["cpi1"]


def test_backward_policy_argmax(dev):
    """The drop-in maxent.local_action_probabilities runs the backward pass in
    numpy's own floating-point order (irlmx_backward_maxent_numpy_order), so the
    policy -- and with it every argmax, the 1-ulp near-ties of the unit-reward
    cases included -- is bit-identical to the reference's output."""
    import maxent as M
    for name, P, term, r, ref in _pinned_backward_cases():
        pi = M.local_action_probabilities(P, term, r)
        assert np.array_equal(pi, ref), (name, np.max(np.abs(pi - ref)))
        got, want = np.argmax(pi, axis=1), np.argmax(ref, axis=1)
        assert np.array_equal(got, want), (name, _argmax_report(got, want))


def test_numpy_order_all_layouts_and_overflow(dev, monkeypatch):
    """ops.backward_maxent_numpy_order on the STENCIL5, ELL and DENSE layouts
    against the reference's output bit for bit, every maxent_small case: the
    overflowing ones give the reference's NaN pattern (no rescaling), and the
    drop-in then reruns them rescaled unless IRLMX_REFERENCE_OVERFLOW=1."""
    import maxent as M
    from irlmx import DeviceMDP, ops
    z = load_golden("maxent_small")
    for c in [str(n) for n in z["names"]]:
        size = int(z[c + "__size"])
        n = size * size
        P = O.icy_gridworld_table(size, float(z[c + "__p_slip"]))
        term = [int(t) for t in z[c + "__terminal"]]
        ref = z[c + "__pi"]
        tm = ops.terminal_mask(term, n, device=dev)
        er = np.exp(z[c + "__reward"])
        for layout in ("stencil", "ell", "dense"):
            mdp = DeviceMDP.from_dense(P, device=dev, layout=layout)
            pi = ops.backward_maxent_numpy_order(mdp, er, tm)[0].cpu().numpy()
            assert np.array_equal(pi, ref, equal_nan=True), (c, layout)
        if not np.isfinite(ref).all():
            monkeypatch.setenv("IRLMX_REFERENCE_OVERFLOW", "1")
            assert np.array_equal(M.local_action_probabilities(P, term, z[c + "__reward"]), ref, equal_nan=True)
            monkeypatch.delenv("IRLMX_REFERENCE_OVERFLOW")
            if term:   # rescaled rerun: the oracle's ratio-exact rescaled pass
                pi = M.local_action_probabilities(P, term, z[c + "__reward"])
                ro = O.backward_maxent(P, term, z[c + "__reward"], rescale=True)
                assert np.isfinite(pi).all() and np.max(np.abs(pi - ro)) <= 1e-8 * np.max(np.abs(ro)), c


def test_numpy_order_generic_and_batched(dev):
    """Non-grid MDPs (tests/golden/generic.npz: sparse, dense and five-action
    tables, S = 20 / 12 / 40) against the C restatement of numpy's order, and a
    batch of instances with per-instance tables and rewards equal to single calls."""
    from irlmx import DeviceMDP, ops
    g = load_golden("generic")
    for c in [str(n) for n in g["names"]]:
        P = g[c + "__P"]
        term = [int(t) for t in g[c + "__terminal"]]
        r = g[c + "__reward"]
        ref = O.backward_maxent_blas_order(P, term, r)
        assert np.array_equal(ref, O.backward_maxent(P, term, r), equal_nan=True), c   # numpy itself, this host
        for layout in ("ell", "dense"):
            mdp = DeviceMDP.from_dense(P, device=dev, layout=layout)
            pi = ops.backward_maxent_numpy_order(mdp, np.exp(r), ops.terminal_mask(term, P.shape[0], device=dev))
            assert np.array_equal(pi[0].cpu().numpy(), ref, equal_nan=True), (c, layout)
    size, B = 9, 3
    n = size * size
    slips = [0.1, 0.2, 0.35]
    rng = np.random.default_rng(4)
    r = rng.uniform(-0.5, 0.3, (B, n))
    mdp = DeviceMDP.icy_gridworld(size, slips, device=dev)
    pi = ops.backward_maxent_numpy_order(mdp, np.exp(r), ops.terminal_mask([n - 1], n, batch=B, device=dev))
    for b in range(B):
        ref = O.backward_maxent_blas_order(O.icy_gridworld_table(size, slips[b]), [n - 1], r[b])
        assert np.array_equal(pi[b].cpu().numpy(), ref, equal_nan=True), b


def test_causal_policy_argmax(dev):
    """The drop-in local_causal_action_probabilities sums every P_a . v in numpy's
    order (irlmx_soft_backward_numpy_order) and evaluates exp / log as numpy's
    AVX512_SKX loops do (np_exp / np_log, csrc/common.h), so the policy is
    bit-identical to the reference's output -- the mirror-symmetric ties of the
    unit-reward cases, decided in the last bit, included -- with identical sweep
    counts, on every layout."""
    import maxent as M
    from irlmx import DeviceMDP, ops
    for name, P, term, r, g, ref in _pinned_causal_cases():
        pi = M.local_causal_action_probabilities(P, term, r, g)
        assert np.array_equal(pi, ref), (name, np.max(np.abs(pi - ref)), int((pi != ref).sum()))
        got, want = np.argmax(pi, axis=1), np.argmax(ref, axis=1)
        assert np.array_equal(got, want), (name, _argmax_report(got, want))
        _, _, ks_ref = O.soft_backward(P, term, r, g)
        for layout in ("stencil", "ell", "dense"):
            mdp = DeviceMDP.from_dense(P, device=dev, layout=layout)
            p2, _, ks, st = ops.soft_backward(mdp, r, O.terminal_reward(term, P.shape[0]), g, numpy_order=True)
            assert int(ks[0]) == ks_ref and int(st[0]) == 0, (name, layout)
            assert torch.equal(p2[0].cpu(), torch.as_tensor(pi)), (name, layout)   # same arithmetic, any layout


def test_value_iteration_numpy_order_bit_identical(dev):
    """solver.value_iteration / stochastic_value_iteration run in numpy's order:
    values and sweep counts bit-identical to the reference's output for every
    golden VI case (5x5 / 16x16, max and average, det4, config 1, the non-grid
    tables on the ELL and DENSE layouts), and to the C restatement
    (oracle/blas_order.c) at 32x32 and 64x64 with random rewards."""
    import solver as S
    from irlmx import DeviceMDP, ops
    z = load_golden("vi")
    for c in [str(n) for n in z["names"]]:
        if c.startswith("det"):
            continue
        P = O.icy_gridworld_table(int(z[c + "__size"]), 0.2)
        fn = S.stochastic_value_iteration if bool(z[c + "__average"]) else S.value_iteration
        v = fn(P, z[c + "__reward"], float(z[c + "__discount"]))
        assert np.array_equal(v, z[c + "__value"]), c
    assert np.array_equal(S.value_iteration(O.gridworld_table(4), z["det4__reward"], 0.5), z["det4__value"])
    z1 = load_golden("config1")
    assert np.array_equal(S.value_iteration(z1["p_transition"], z1["reward"], 0.7), z1["value"])
    g = load_golden("generic")
    for c in [str(n) for n in g["names"]]:
        P, r = g[c + "__P"], g[c + "__reward"]
        for layout in ("ell", "dense"):
            mdp = DeviceMDP.from_dense(P, device=dev, layout=layout)
            for avg, key in ((False, "__v"), (True, "__va")):
                v, k, _ = ops.value_iteration(mdp, r, 0.9, average=avg, numpy_order=True)
                assert np.array_equal(v[0].cpu().numpy(), g[c + key]), (c, layout, avg)
    rng = np.random.default_rng(9)
    for size in (32, 64):
        P = O.icy_gridworld_table(size, 0.25)
        r = rng.uniform(-1.0, 1.0, size * size)
        mdp = DeviceMDP.icy_gridworld(size, 0.25, device=dev)
        for avg in (False, True):
            ref, kr = O.value_iteration_blas_order(P, r, 0.95, average=avg)
            v, k, _ = ops.value_iteration(mdp, r, 0.95, average=avg, numpy_order=True)
            assert int(k[0]) == kr and np.array_equal(v[0].cpu().numpy(), ref), (size, avg)


def test_forward_numpy_order_bit_identical(dev):
    """irlmx_forward_svf_numpy_order (maxent.py:105-114 in numpy's order): from
    the reference's own policies, SVF and sweep counts bit-identical to the
    reference's output for every maxent_small case -- the 11,858,933-sweep s8_unif
    case included, which the tiled shapes may end a few sweeps early or late --,
    config 1's svf1 / csvf1 and the non-grid tables; STENCIL5, ELL and DENSE
    layouts (ELL and DENSE skip the 11.9M-sweep case)."""
    import maxent as M
    from irlmx import DeviceMDP, ops
    z = load_golden("maxent_small")
    for c in [str(n) for n in z["names"]]:
        size = int(z[c + "__size"])
        n = size * size
        P = O.icy_gridworld_table(size, float(z[c + "__p_slip"]))
        term = [int(t) for t in z[c + "__terminal"]]
        tm = ops.terminal_mask(term, n, device=dev)
        for layout in ("stencil", "ell", "dense"):
            if layout != "stencil" and int(z[c + "__k_f"]) > 100_000:
                continue   # (the general kernel re-reads its entries every sweep: ~15 us per sweep)
            mdp = DeviceMDP.from_dense(P, device=dev, layout=layout)
            svf, k, st = ops.forward_svf(mdp, z[c + "__p0"], tm, z[c + "__pi"], numpy_order=True)
            assert int(k[0]) == int(z[c + "__k_f"]), (c, layout, int(k[0]))
            assert np.array_equal(svf[0].cpu().numpy(), z[c + "__svf"], equal_nan=True), (c, layout)
    z1 = load_golden("config1")
    P = z1["p_transition"]
    assert np.array_equal(M.expected_svf_from_policy(P, z1["p_initial"], [24], z1["pi1"]), z1["svf1"])
    assert np.array_equal(M.expected_svf_from_policy(P, z1["p_initial"], [24], z1["cpi1"]), z1["csvf1"])
    assert np.array_equal(M.compute_expected_svf(P, z1["p_initial"], [24], np.ones(25)), z1["svf1"])
    g = load_golden("generic")
    for c in [str(n) for n in g["names"]]:
        P = g[c + "__P"]
        S = P.shape[0]
        term = [int(t) for t in g[c + "__terminal"]]
        for layout in ("ell", "dense"):
            mdp = DeviceMDP.from_dense(P, device=dev, layout=layout)
            svf, k, _ = ops.forward_svf(mdp, g[c + "__p0"], ops.terminal_mask(term, S, device=dev), g[c + "__pi"],
                                        numpy_order=True)
            assert int(k[0]) == int(g[c + "__k_f"]), (c, layout)
            assert np.array_equal(svf[0].cpu().numpy(), g[c + "__svf"]), (c, layout)


def test_config1_irl_bit_identical(dev):
    """BASELINE config 1 (src/main.py) through the drop-in: maxent.irl's 375
    steps reproduce the reference's recovered reward bit for bit (backward and
    forward in numpy's order, the caller's numpy optimiser on the host), and
    irl_causal its 419 steps too (soft VI with numpy's exp / log, np_exp /
    np_log)."""
    import maxent as M
    from conftest import unpack_trajectories
    z = load_golden("config1")
    tjs = unpack_trajectories(z["traj_flat"], z["traj_lens"])
    opt = O.ExpSga(lr=O.linear_decay(0.2))
    r = M.irl(z["p_transition"], np.identity(25), [24], tjs, opt, O.Constant(1.0))
    assert opt.k == int(z["irl_steps"]) == 375
    assert np.array_equal(r, z["reward_maxent"]), np.max(np.abs(r - z["reward_maxent"]))
    opt = O.ExpSga(lr=O.linear_decay(0.2))
    r = M.irl_causal(z["p_transition"], np.identity(25), [24], tjs, opt, O.Constant(1.0), 0.7)
    assert opt.k == int(z["causal_steps"]) == 419
    assert np.array_equal(r, z["reward_causal"]), np.max(np.abs(r - z["reward_causal"]))


@pytest.mark.parametrize("size", [23, 31, 32])
def test_forward_numpy_order_two_targets_per_lane(dev, size):
    """The register-cached numpy-order forward at one (23x23) and two (31x31,
    32x32: 961 / 1024 states, S % 4 = 1 and 0) targets per lane against the C
    restatement of numpy's order (oracle/blas_order.c), a capped 200-sweep run
    from a random policy: bit for bit."""
    from irlmx import DeviceMDP, ops
    n = size * size
    P = O.icy_gridworld_table(size, 0.2)
    rng = np.random.default_rng(size)
    pi = rng.uniform(0.1, 1.0, (n, 4))
    pi /= pi.sum(axis=1, keepdims=True)
    p0 = np.zeros(n)
    p0[rng.integers(0, n, 5)] = 0.2
    term = [n - 1, n // 2]
    ref, kr = O.forward_svf_blas_order(P, p0, term, pi, max_iter=200)
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    svf, k, _ = ops.forward_svf(mdp, p0, ops.terminal_mask(term, n, device=dev), pi, max_iter=200, numpy_order=True)
    assert int(k[0]) == kr == 200
    assert np.array_equal(svf[0].cpu().numpy(), ref)


@pytest.mark.parametrize("size", [16, 23])
def test_backward_numpy_order_cached_against_restatement(dev, size):
    """The register-cached numpy-order backward (one state per lane at 16x16,
    two at 23x23 = 529 states, S % 4 = 1: the last row's rounded-product lanes
    and the fused last column) against the C restatement of numpy's order, with
    rewards near -ln 4 so that the 2 S sweeps neither overflow nor underflow:
    bit for bit."""
    from irlmx import DeviceMDP, ops
    n = size * size
    r = -np.log(4.0) + np.random.default_rng(size).uniform(-0.05, 0.05, n)
    P = O.icy_gridworld_table(size, 0.2)
    ref = O.backward_maxent_blas_order(P, [n - 1], r)
    assert np.isfinite(ref).all()
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    pi = ops.backward_maxent_numpy_order(mdp, np.exp(r), ops.terminal_mask([n - 1], n, device=dev))
    assert np.array_equal(pi[0].cpu().numpy(), ref)


def test_backward_numpy_order_64x64_against_restatement(dev, monkeypatch):
    """64x64 (S = 4096, the largest model the drop-ins run in numpy's order):
    the device's numpy-order backward against the C restatement of numpy's
    order (its sparse form, oracle/blas_order.c, pinned to the dense form and to
    np.dot at S = 4096 -- both NBMAX = 2048 column blocks -- in
    tests/test_oracle_blas_order.py), rewards near -ln 4 so that the 2 S = 8192
    sweeps stay finite: bit for bit, through ops on the device-built table and
    through the drop-in on the uploaded dense table."""
    import maxent as M
    from irlmx import DeviceMDP, ops
    size = 64
    n = size * size
    r = -np.log(4.0) + np.random.default_rng(64).uniform(-0.05, 0.05, n)
    ref = O.backward_maxent_blas_order_csr(O.icy_gridworld_csr(size, 0.2), [n - 1], r)
    assert np.isfinite(ref).all()
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    pi = ops.backward_maxent_numpy_order(mdp, np.exp(r), ops.terminal_mask([n - 1], n, device=dev))
    assert np.array_equal(pi[0].cpu().numpy(), ref), np.max(np.abs(pi[0].cpu().numpy() - ref))
    # (the drop-in's default numpy-order scope is 1024 states, ops.numpy_order_default)
    assert not ops.numpy_order_default(mdp)
    monkeypatch.setenv("IRLMX_NUMPY_ORDER_MAX", "4096")
    got = M.local_action_probabilities(O.icy_gridworld_table(size, 0.2), [n - 1], r)
    assert np.array_equal(got, ref)
    assert np.array_equal(np.argmax(got, axis=1), np.argmax(ref, axis=1))


class IcyWorld64:
    """The reference IcyGridWorld(64, 0.2) API the solver drop-ins use: size,
    actions, n_states / n_actions, state_index_transition, p_transition (the
    oracle's table, sha256-equal to the reference builder's: tests/golden/c2_64.npz,
    test_oracle_golden.py::test_c2_64_fixture_table)."""

    def __init__(self):
        self.size, self.n_states, self.n_actions = 64, 4096, 4
        self.actions = O.ACTIONS
        self.p_transition = O.icy_gridworld_table(64, 0.2)

    def state_index_transition(self, s, a):
        return O.intended_successor(self.size, s, a)


def test_config2_drop_ins_against_reference(dev):
    """BASELINE config 2's world (64x64 IcyGridWorld, A = 4, S = 4096) through the
    drop-ins under their DEFAULT settings, against the reference run on the same
    table with one BLAS thread (tests/golden/c2_64.npz, tools/gen_golden.py
    c2_64): theta = 1 (mirror-symmetric exact ties, decided in the last bit) and
    a seeded uniform theta.

    * solver.value_iteration / stochastic_value_iteration (solver.py:9-104),
      discounts 0.7 / 0.9: values bit-identical, sweep counts identical;
      solver.optimal_policy_from_value and solver.optimal_policy
      (solver.py:107-152): np.array_equal with the reference's greedy policy.
    * maxent.local_causal_action_probabilities (maxent.py:279-341): soft-VI
      sweep count identical, policy bit-identical (numpy's order for P_a . v,
      numpy's exp / log: np_exp / np_log), so np.array_equal argmax -- at
      theta = 1 too, whose ~2,200 mirror-symmetric near-ties (710 exact) are
      decided by the last bits of ~700 sweeps of exp / log."""
    import maxent as M
    import solver as S
    from irlmx import ops
    z = load_golden("c2_64")
    world = IcyWorld64()
    P = world.p_transition
    n = world.n_states
    mdp = S._model(P)
    assert ops.numpy_order_default(mdp, "value_iteration") and ops.numpy_order_default(mdp, "soft_backward")
    names = [str(c) for c in z["names"]]
    assert len(names) == 12
    for c in names:
        r = z[c.split("_")[0] + "__reward"]
        g = float(z[c + "__discount"])
        if "_soft_" in c:
            ref = z[c + "__pi"]
            pi = M.local_causal_action_probabilities(P, [n - 1], r, g)
            got, want = np.argmax(pi, axis=1), np.argmax(ref, axis=1)
            assert np.array_equal(pi, ref), (c, np.max(np.abs(pi - ref)), int((pi != ref).sum()))
            assert np.array_equal(got, want), (c, _argmax_report(got, want))
            _, _, ks, st = ops.soft_backward(mdp, r, O.terminal_reward([n - 1], n), g, numpy_order=True)
            assert int(ks[0]) == int(z[c + "__k_s"]) and int(st[0]) == 0, (c, int(ks[0]))
            top = np.sort(ref, axis=1)
            near = int(((top[:, -1] - top[:, -2]) <= 1e-14 * top[:, -1]).sum())
            print(f"[c2_64] {c}: {int(ks[0])} sweeps; policy bit-identical, argmax equal at all {n} states "
                  f"({near} of them tied within 1e-14)", flush=True)
            continue
        avg = bool(z[c + "__average"])
        fn = S.stochastic_value_iteration if avg else S.value_iteration
        v = fn(P, r, g)
        assert np.array_equal(v, z[c + "__value"]), (c, np.max(np.abs(v - z[c + "__value"])))
        _, k, _ = ops.value_iteration(mdp, r, g, average=avg, numpy_order=True)
        assert int(k[0]) == int(z[c + "__k"]), (c, int(k[0]))
        pol = S.optimal_policy_from_value(world, v)
        assert np.array_equal(pol, z[c + "__opt_policy"]), (c, _argmax_report(pol, z[c + "__opt_policy"]))
        if not avg:
            pol2 = S.optimal_policy(world, r, g)
            assert np.array_equal(pol2, z[c + "__opt_policy"]), (c, _argmax_report(pol2, z[c + "__opt_policy"]))
        print(f"[c2_64] {c}: values bit-identical, {int(k[0])} sweeps, greedy policy equal", flush=True)
