"""Pin the CPU oracle against golden vectors produced by the reference itself.

The fixtures under tests/golden/ come from tools/gen_golden.py, which imports
the reference (narendasan/irl-maxent, src/) read-only.  The oracle evaluates
the same numpy statements in the same order, so these checks are bit-exact
(``np.array_equal``) including the sweep counts of every fixed-point loop.
"""

import hashlib

import numpy as np
import pytest

import maxent_oracle as O
from conftest import load_golden, unpack_trajectories

# forward passes longer than this are skipped on CPU (the oracle needs minutes)
CPU_SWEEP_BUDGET = 200_000


def _cases(z):
    return [str(n) for n in z["names"]]


def test_world_tables_bit_exact():
    z = load_golden("worlds")
    for size, p_slip in ((5, 0.2), (8, 0.1), (8, 0.3), (3, 0.2)):
        assert np.array_equal(O.icy_gridworld_table(size, p_slip), z[f"icy_{size}_{p_slip}"])
    assert np.array_equal(O.gridworld_table(5), z["det_5"])
    h = hashlib.sha256(np.ascontiguousarray(O.icy_gridworld_table(16, 0.2)).tobytes()).hexdigest()
    assert h == str(z["icy_16_0.2_sha256"])
    h = hashlib.sha256(np.ascontiguousarray(O.gridworld_table(16)).tobytes()).hexdigest()
    assert h == str(z["det_16_sha256"])


def test_config1_pipeline_pieces():
    z = load_golden("config1")
    P = z["p_transition"]
    assert np.array_equal(P, O.icy_gridworld_table(5, 0.2))
    v, k = O.value_iteration(P, z["reward"], 0.7)
    assert np.array_equal(v, z["value"]) and k == int(z["vi_sweeps"])
    assert np.array_equal(O.optimal_policy_from_value(5, v), z["opt_policy"])
    assert np.array_equal(O.stochastic_policy_from_value(5, v, w=lambda x: x ** 5), z["policy"])
    tjs = unpack_trajectories(z["traj_flat"], z["traj_lens"])
    feats = np.identity(25)
    assert np.array_equal(O.feature_expectation(feats, tjs), z["e_features"])
    assert np.array_equal(O.initial_probabilities(25, tjs), z["p_initial"])
    term = [int(t) for t in z["terminal"]]
    pi = O.backward_maxent(P, term, np.ones(25))
    assert np.array_equal(pi, z["pi1"])
    assert np.array_equal(O.backward_maxent(P, term, np.ones(25), rescale=True), z["pi1"])
    svf, k = O.forward_svf(P, z["p_initial"], term, pi)
    assert np.array_equal(svf, z["svf1"]) and k == int(z["k_f1"])
    cpi, _, ks = O.soft_backward(P, term, np.ones(25), 0.7)
    assert np.array_equal(cpi, z["cpi1"]) and ks == int(z["k_s1"])
    csvf, k = O.forward_svf(P, z["p_initial"], term, cpi)
    assert np.array_equal(csvf, z["csvf1"]) and k == int(z["k_cf1"])


def test_config1_irl_full_run():
    z = load_golden("config1")
    P = z["p_transition"]
    tjs = unpack_trajectories(z["traj_flat"], z["traj_lens"])
    term = [int(t) for t in z["terminal"]]
    r, steps = O.irl(P, np.identity(25), term, tjs, O.ExpSga(lr=O.linear_decay(0.2)), O.Constant(1.0))
    assert steps == int(z["irl_steps"])
    assert np.array_equal(r, z["reward_maxent"])


@pytest.mark.slow
def test_config1_irl_causal_full_run():
    z = load_golden("config1")
    P = z["p_transition"]
    tjs = unpack_trajectories(z["traj_flat"], z["traj_lens"])
    term = [int(t) for t in z["terminal"]]
    r, steps = O.irl_causal(P, np.identity(25), term, tjs, O.ExpSga(lr=O.linear_decay(0.2)),
                            O.Constant(1.0), 0.7)
    assert steps == int(z["causal_steps"])
    assert np.array_equal(r, z["reward_causal"])


def test_maxent_small_cases():
    z = load_golden("maxent_small")
    for c in _cases(z):
        P = O.icy_gridworld_table(int(z[c + "__size"]), float(z[c + "__p_slip"]))
        term = [int(t) for t in z[c + "__terminal"]]
        with np.errstate(all="ignore"):
            pi = O.backward_maxent(P, term, z[c + "__reward"])
        assert np.array_equal(pi, z[c + "__pi"], equal_nan=True), c
        if np.isfinite(pi).all():
            # power-of-two rescaling leaves the ratio bit-identical where finite
            assert np.array_equal(O.backward_maxent(P, term, z[c + "__reward"], rescale=True), pi), c
        if int(z[c + "__k_f"]) > CPU_SWEEP_BUDGET:
            continue
        with np.errstate(all="ignore"):
            svf, k = O.forward_svf(P, z[c + "__p0"], term, pi)
        assert np.array_equal(svf, z[c + "__svf"], equal_nan=True), c
        assert k == int(z[c + "__k_f"]), c


def test_value_iteration_cases():
    z = load_golden("vi")
    for c in _cases(z):
        size = int(z[c + "__size"])
        P = O.icy_gridworld_table(size, 0.2)
        avg = bool(z[c + "__average"])
        v, k = O.value_iteration(P, z[c + "__reward"], float(z[c + "__discount"]), average=avg)
        assert np.array_equal(v, z[c + "__value"]) and k == int(z[c + "__k"]), c
        if not avg:
            assert np.array_equal(O.optimal_policy_from_value(size, v), z[c + "__opt_policy"])
            sp = O.stochastic_policy_from_value(size, v, w=lambda x: np.exp(x))
            assert np.array_equal(sp, z[c + "__stoch_policy"])
    P = O.gridworld_table(4)
    v, k = O.value_iteration(P, z["det4__reward"], 0.5)
    assert np.array_equal(v, z["det4__value"]) and k == int(z["det4__k"])
    assert np.array_equal(O.optimal_policy_from_value(4, v), z["det4__opt_policy"])


def test_generic_mdps():
    z = load_golden("generic")
    for c in _cases(z):
        P = z[c + "__P"]
        term = [int(t) for t in z[c + "__terminal"]]
        r, p0 = z[c + "__reward"], z[c + "__p0"]
        pi = O.backward_maxent(P, term, r)
        assert np.array_equal(pi, z[c + "__pi"]), c
        svf, k = O.forward_svf(P, p0, term, pi)
        assert np.array_equal(svf, z[c + "__svf"]) and k == int(z[c + "__k_f"]), c
        cpi, _, ks = O.soft_backward(P, term, r, 0.8)
        assert np.array_equal(cpi, z[c + "__cpi"]) and ks == int(z[c + "__k_s"]), c
        v, kv = O.value_iteration(P, r, 0.9)
        assert np.array_equal(v, z[c + "__v"]) and kv == int(z[c + "__k_v"]), c
        va, kva = O.value_iteration(P, r, 0.9, average=True)
        assert np.array_equal(va, z[c + "__va"]) and kva == int(z[c + "__k_va"]), c


def test_causal_small_cases():
    z = load_golden("causal_small")
    for c in _cases(z):
        size = int(z[c + "__size"])
        P = O.icy_gridworld_table(size, 0.2)
        term = [int(t) for t in z[c + "__terminal"]]
        pi, _, ks = O.soft_backward(P, term, z[c + "__reward"], float(z[c + "__discount"]))
        assert np.array_equal(pi, z[c + "__pi"]) and ks == int(z[c + "__k_s"]), c
        if size <= 16:
            svf, k = O.forward_svf(P, z[c + "__p0"], term, pi)
            assert np.array_equal(svf, z[c + "__svf"]) and k == int(z[c + "__k_f"]), c
    P = O.icy_gridworld_table(5, 0.2)
    pi, _, ks = O.soft_backward(P, z["phi_vec__phi"], np.ones(25), 0.8)
    assert np.array_equal(pi, z["phi_vec__pi"]) and ks == int(z["phi_vec__k_s"])


def test_sparse_oracle_matches_dense():
    """The sparse-operand restatement (used at 128x128 in test_gpu_full_size.py)
    builds the same table values as the dense oracle (bit for bit) and runs the
    same statements: backward and forward agree to rounding, sweep counts equal."""
    for size, slip in ((5, 0.2), (9, 0.1), (16, 0.3)):
        P = O.icy_gridworld_table(size, slip)
        mats = O.icy_gridworld_csr(size, slip)
        assert np.array_equal(np.stack([m.toarray() for m in mats], axis=2), P), size
    rng = np.random.default_rng(3)
    for size in (5, 12):
        n = size * size
        P = O.icy_gridworld_table(size, 0.2)
        mats = O.icy_gridworld_csr(size, 0.2)
        r = rng.uniform(0.0, 1.0, n)
        pi = O.backward_maxent(P, [n - 1], r, rescale=True)
        pi_s = O.backward_maxent_csr(mats, [n - 1], r)
        assert np.max(np.abs(pi_s - pi)) <= 1e-13 * np.max(pi)
        p0 = np.zeros(n)
        p0[0] = 1.0
        d, k = O.forward_svf(P, p0, [n - 1], pi)
        d_s, k_s = O.forward_svf_csr(mats, p0, [n - 1], pi)
        assert k == k_s and np.max(np.abs(d_s - d)) <= 1e-12 * np.max(d)


def test_sparse_soft_backward_matches_dense():
    """soft_backward_csr (the config-2 stay-variant check in test_gpu_full_size.py)
    against the dense restatement, which the causal golden vectors pin: the
    same sweep count, policy and values to rounding -- including a 5-action
    table (the four moves plus "stay")."""
    import scipy.sparse as sp
    rng = np.random.default_rng(10)
    for size, stay in ((5, False), (12, False), (12, True)):
        n = size * size
        mats = O.icy_gridworld_csr(size, 0.2) + ([sp.identity(n, format="csr")] if stay else [])
        P = np.stack([m.toarray() for m in mats], axis=2)
        r = rng.uniform(0.0, 1.0, n)
        pi, v, k = O.soft_backward(P, [n - 1], r, 0.7)
        pi_s, v_s, k_s = O.soft_backward_csr(mats, [n - 1], r, 0.7)
        assert k == k_s, (size, stay)
        assert np.max(np.abs(pi_s - pi)) <= 1e-12 * np.max(pi)
        assert np.max(np.abs(v_s - v)) <= 1e-12 * np.max(np.abs(v))


def test_sparse_value_iteration_matches_dense():
    rng = np.random.default_rng(9)
    for size in (5, 16):
        n = size * size
        P = O.icy_gridworld_table(size, 0.2)
        mats = O.icy_gridworld_csr(size, 0.2)
        r = rng.uniform(0.0, 1.0, n)
        for avg in (False, True):
            v, k = O.value_iteration(P, r, 0.9, average=avg)
            vs, ks = O.value_iteration_csr(mats, r, 0.9, average=avg)
            assert k == ks and np.max(np.abs(vs - v)) <= 1e-12 * np.max(np.abs(v))


def test_full_size_fixtures_consistent():
    """The converged full-size fixtures (tools/gen_full_fixtures.py) are what the
    oracle's own loops produce: their inputs regenerate bit for bit (bench slips,
    demonstrations from the oracle's STENCIL5 table, the seeded dense MDP), and a
    short re-run of the CSR irl restatement on a 16x16 version of the bench
    workload matches the dense oracle's loop."""
    import numpy as np
    from irlmx import demos
    for cfg, size, total in (("c2", 64, 1), ("c3", 128, 64), ("c4", 256, 32), ("c5", 128, 1)):
        z = load_golden(f"full_{cfg}")
        b = int(z["instances"][0])
        slip = 0.1 + 0.2 * b / total
        assert float(z[f"{b}__slip"]) == slip
        n = size * size
        rv = O.stencil_row_val(O.icy_gridworld_csr(size, slip), size)
        e_f, p0, lens = demos.sample(rv, size, [n - 1], 0, n=200, seed=1234 + b)
        assert np.array_equal(e_f, z[f"{b}__e_f"]) and np.array_equal(p0, z[f"{b}__p0"])
        # no demonstration of the bench workloads is cut: under the former cap of
        # 64 * size steps (which produced the fixtures) every trajectory reached
        # the terminal state, so the uncapped sampler regenerates them unchanged
        cap = 64 * size
        _, _, lens_c, cut = demos.sample(rv, size, [n - 1], 0, n=200, seed=1234 + b, max_len=cap,
                                         with_truncated=True)
        assert cut == 0 and np.array_equal(lens_c, lens) and int(lens.max()) < cap, (cfg, int(lens.max()))
    z = load_golden("dense2048")
    P, r, term, p0 = O.random_dense_mdp()
    assert np.array_equal(np.array([P.sum(), P[::7, ::5, :].sum(), P[-1, -1, -1]]), z["P_check"])
    assert np.array_equal(r, z["reward"])
    # the CSR irl steps restate the dense loop (maxent.py:240-252) on a small grid
    size, n = 16, 256
    mats = O.icy_gridworld_csr(size, 0.15)
    e_f, p0, _ = demos.sample(O.stencil_row_val(mats, size), size, [n - 1], 0, n=50, seed=7)
    res = O.irl_steps_csr(mats, e_f, p0, [n - 1], 3)
    Pd = O.icy_gridworld_table(size, 0.15)
    theta = np.ones(n)
    for k in range(3):
        pi = O.backward_maxent(Pd, [n - 1], theta, rescale=True)
        svf, kf = O.forward_svf(Pd, p0, [n - 1], pi)
        theta = theta * np.exp(0.2 / (1 + k) * (e_f - svf))
        assert kf == res["k_f"][k]
        assert np.max(np.abs(theta - res["theta"][k])) <= 1e-12 * np.max(np.abs(theta))


def test_c2_64_fixture_table():
    """tests/golden/c2_64.npz (config 2's world through the reference, one BLAS
    thread) was made on the reference builder's table, which equals the oracle's
    64x64 IcyGridWorld byte for byte; value iteration in numpy's order restated
    in C (oracle/blas_order.c) reproduces the reference's values and sweep counts
    bit for bit at S = 4096 (both NBMAX = 2048 column blocks), and the CSR
    restatement within 1e-12 with the same sweep counts."""
    z = load_golden("c2_64")
    assert int(z["size"]) == 64 and float(z["p_slip"]) == 0.2
    P = O.icy_gridworld_table(64, 0.2)
    assert hashlib.sha256(np.ascontiguousarray(P).tobytes()).hexdigest() == str(z["P_sha256"])
    mats = O.icy_gridworld_csr(64, 0.2)
    for c in ("ones_g7_max", "unif_g7_avg", "unif_g9_max"):
        r = z[c.split("_")[0] + "__reward"]
        g, avg = float(z[c + "__discount"]), bool(z[c + "__average"])
        v, k = O.value_iteration_blas_order(P, r, g, average=avg)
        assert k == int(z[c + "__k"]) and np.array_equal(v, z[c + "__value"]), c
        vs, ks = O.value_iteration_csr(mats, r, g, average=avg)
        assert ks == k and np.max(np.abs(vs - v)) <= 1e-12 * np.max(np.abs(v)), c
    # the reference's greedy policy from its own values (solver.py:107-124)
    for c in ("ones_g9_max", "unif_g7_max"):
        assert np.array_equal(O.optimal_policy_from_value(64, z[c + "__value"]), z[c + "__opt_policy"]), c


def test_demos_truncation_reported():
    """irlmx.demos.sample samples until terminal like the reference
    (trajectory.py:76); a cap that cuts trajectories raises, or is counted."""
    import numpy as np
    import pytest
    from irlmx import demos
    size, n = 8, 64
    rv = O.stencil_row_val(O.icy_gridworld_csr(size, 0.2), size)
    _, _, lens = demos.sample(rv, size, [n - 1], 0, n=20, seed=3)
    assert int(lens.min()) >= 2 * (size - 1)          # Manhattan distance from state 0 to the goal
    with pytest.raises(demos.TruncatedDemonstrations):
        demos.sample(rv, size, [n - 1], 0, n=20, seed=3, max_len=5)
    e_f, _, lens5, cut = demos.sample(rv, size, [n - 1], 0, n=20, seed=3, max_len=5, on_truncate="allow",
                                      with_truncated=True)
    assert cut == 20 and int(lens5.max()) == 5 and abs(e_f.sum() - 6.0) < 1e-12   # 5 steps + the cut state


def _optimizer_cases():
    z = load_golden("optimizers")
    make = {
        "sga_power": (lambda: O.Sga(lr=O.power_decay(lr0=0.2, power=2)), lambda: O.Constant(1.0)),
        "sga_linear": (lambda: O.Sga(lr=O.linear_decay(lr0=0.2)), lambda: O.Constant(1.0)),
        "expsga_expdecay": (lambda: O.ExpSga(lr=O.exponential_decay(lr0=0.2, decay_rate=0.01)),
                            lambda: O.Constant(1.0)),
        "norm_expsga": (lambda: O.NormalizeGrad(O.ExpSga(lr=O.linear_decay(lr0=0.2))), lambda: O.Constant(1.0)),
        "norm1_sga": (lambda: O.NormalizeGrad(O.Sga(lr=O.power_decay(lr0=0.5, decay_steps=2, power=1.5)), ord=1),
                      lambda: O.Constant(1.0)),
        "expsga_normalize_uniform": (lambda: O.ExpSga(lr=O.linear_decay(lr0=0.2), normalize=True),
                                     lambda: O.Uniform(0.5, 1.5)),
        "causal_norm1_sga": (lambda: O.NormalizeGrad(O.Sga(lr=O.power_decay(lr0=0.5, decay_steps=2, power=1.5)),
                                                     ord=1), lambda: O.Constant(1.0)),
    }
    assert sorted(make) == sorted(str(n) for n in z["names"])
    return z, make


@pytest.mark.slow
def test_oracle_optimizers_match_reference():
    """The oracle's Sga, NormalizeGrad, ExpSga(normalize), power / exponential
    decay and Uniform (optimizer.py:61-398) reproduce the reference's full irl /
    irl_causal runs of tests/golden/optimizers.npz (tools/gen_golden.py) bit for bit."""
    z, make = _optimizer_cases()
    c1 = load_golden("config1")
    tjs = unpack_trajectories(c1["traj_flat"], c1["traj_lens"])
    P, feats = c1["p_transition"], np.identity(25)
    for name in ("sga_power", "norm1_sga", "expsga_normalize_uniform", "causal_norm1_sga"):
        mk_opt, mk_init = make[name]
        np.random.seed(7)
        assert np.array_equal(mk_init()(25), z[name + "__theta0"]), name
        np.random.seed(7)
        if name.startswith("causal"):
            r, k = O.irl_causal(P, feats, [24], tjs, mk_opt(), mk_init(), 0.7)
        else:
            r, k = O.irl(P, feats, [24], tjs, mk_opt(), mk_init())
        assert k == int(z[name + "__steps"]) and np.array_equal(r, z[name + "__reward"]), name
