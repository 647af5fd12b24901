#!/usr/bin/env python
"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's own modules (no file of the
reference is modified or copied; bytecode writing is disabled) and records
inputs and outputs as small .npz files.  The GPU box never sees the reference:
tests there read only these fixtures.

Process-local shim: ``np.float = float``.  The reference's causal path uses the
alias removed in numpy 1.24 (maxent.py:314, 336); setting it in this process
restores the reference's intended behaviour without touching its files.

Sweep counts: the reference discards the number of fixed-point sweeps it runs.
They are recovered without modifying it by passing ``p_initial`` (forward
pass), ``reward`` (soft VI / VI) as an ndarray subclass that counts the single
``np.add`` each sweep applies to it (maxent.py:110, 329; solver.py:47, 99).

Usage:  python tools/gen_golden.py [--only NAME ...] [--heavy]
"""

import argparse
import hashlib
import os
import sys
import time

import numpy as np

REF_SRC = "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
ORACLE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle")

sys.dont_write_bytecode = True
sys.path.insert(0, REF_SRC)
np.float = float  # shim, see module docstring

import gridworld as W    # noqa: E402  (reference)
import maxent as M       # noqa: E402  (reference)
import optimizer as O    # noqa: E402  (reference)
import solver as S       # noqa: E402  (reference)
import trajectory as T   # noqa: E402  (reference)

sys.path.insert(0, ORACLE_DIR)
import maxent_oracle as ORC  # noqa: E402  (only for the fast 128x128 table build)


class Counted(np.ndarray):
    """ndarray that counts ``np.add`` calls whose first operand is itself."""

    count = 0

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        if ufunc is np.add and method == "__call__" and inputs and inputs[0] is self:
            Counted.count += 1
        args = [np.asarray(x) if isinstance(x, Counted) else x for x in inputs]
        return getattr(ufunc, method)(*args, **kwargs)


def counted(a):
    Counted.count = 0
    return np.asarray(a, dtype=float).view(Counted)


def ref_forward(P, p0, terminal, pi, eps=1e-5):
    c = counted(p0)
    d = M.expected_svf_from_policy(P, c, terminal, pi, eps)
    return np.asarray(d), Counted.count


def ref_soft(P, terminal, r, discount, eps=1e-5):
    c = counted(r)
    pi = M.local_causal_action_probabilities(P, terminal, c, discount, eps)
    n_actions = P.shape[2]
    return np.asarray(pi), Counted.count // n_actions


def ref_vi(P, r, discount, eps=1e-3, average=False):
    c = counted(r)
    fn = S.stochastic_value_iteration if average else S.value_iteration
    v = fn(P, c, discount, eps)
    return np.asarray(v).reshape(-1), Counted.count


class CountingExpSga(O.ExpSga):
    """Reference ExpSga that also counts its steps (outer IRL iterations)."""

    def step(self, grad, *args, **kwargs):
        self.n_steps = getattr(self, "n_steps", 0) + 1
        return super().step(grad, *args, **kwargs)


def pack_trajectories(tjs):
    flat = np.array([tr for t in tjs for tr in t.transitions()], dtype=np.int64)
    lens = np.array([len(t.transitions()) for t in tjs], dtype=np.int64)
    return flat, lens


def save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} B)")


# ---------------------------------------------------------------------------

def gen_config1():
    """G1: the src/main.py pipeline (config 1) with np.random.seed(0)."""
    world = W.IcyGridWorld(size=5, p_slip=0.2)
    reward = np.zeros(world.n_states)
    reward[-1] = 1.0
    reward[8] = 0.65
    terminal = [24]
    value, vi_sweeps = ref_vi(world.p_transition, reward, 0.7)
    value_plain = S.value_iteration(world.p_transition, reward, 0.7)
    assert np.array_equal(value, np.asarray(value_plain).reshape(-1))
    policy = S.stochastic_policy_from_value(world, value_plain, w=lambda x: x ** 5)
    opt_policy = S.optimal_policy_from_value(world, value_plain)
    initial = np.zeros(world.n_states)
    initial[0] = 1.0
    np.random.seed(0)
    tjs = list(T.generate_trajectories(200, world, T.stochastic_policy_adapter(policy),
                                       initial, terminal))
    flat, lens = pack_trajectories(tjs)
    features = W.state_features(world)
    e_features = M.feature_expectation_from_trajectories(features, tjs)
    p_initial = M.initial_probabilities_from_trajectories(world.n_states, tjs)

    # first gradient step intermediates at theta = Constant(1)
    r1 = features.dot(np.ones(world.n_states))
    pi1 = M.local_action_probabilities(world.p_transition, terminal, r1)
    svf1, k_f1 = ref_forward(world.p_transition, p_initial, terminal, pi1)
    cpi1, k_s1 = ref_soft(world.p_transition, terminal, r1, 0.7)
    csvf1, k_cf1 = ref_forward(world.p_transition, p_initial, terminal, cpi1)

    t0 = time.time()
    opt = CountingExpSga(lr=O.linear_decay(lr0=0.2))
    reward_maxent = M.irl(world.p_transition, features, terminal, tjs, opt, O.Constant(1.0))
    irl_steps = opt.n_steps
    t1 = time.time()
    opt = CountingExpSga(lr=O.linear_decay(lr0=0.2))
    reward_causal = M.irl_causal(world.p_transition, features, terminal, tjs, opt,
                                 O.Constant(1.0), 0.7)
    causal_steps = opt.n_steps
    t2 = time.time()
    print(f"config1: irl {irl_steps} steps {t1 - t0:.2f}s, causal {causal_steps} steps {t2 - t1:.2f}s")
    save("config1", p_transition=world.p_transition, reward=reward, terminal=np.array(terminal),
         value=value, vi_sweeps=vi_sweeps, policy=policy, opt_policy=opt_policy,
         traj_flat=flat, traj_lens=lens, e_features=e_features, p_initial=p_initial,
         pi1=pi1, svf1=svf1, k_f1=k_f1, cpi1=cpi1, k_s1=k_s1, csvf1=csvf1, k_cf1=k_cf1,
         reward_maxent=reward_maxent, irl_steps=irl_steps,
         reward_causal=reward_causal, causal_steps=causal_steps,
         t_irl=t1 - t0, t_causal=t2 - t1)


def gen_maxent_small():
    """G2: backward + forward (non-causal) at 5x5, 8x8, 12x12, several thetas/terminals."""
    out = {}
    rng = np.random.default_rng(2)
    cases = []
    for size in (5, 8, 12):
        n = size * size
        cases.append((f"s{size}_ones", size, 0.2, np.ones(n), [n - 1]))
        cases.append((f"s{size}_unif", size, 0.2, rng.uniform(0.0, 1.5, n), [n - 1]))
    cases.append(("s5_neg", 5, 0.2, rng.uniform(0.0, 1.0, 25), [-1]))
    cases.append(("s5_multi", 5, 0.3, rng.uniform(0.0, 1.0, 25), [0, 12, 24]))
    cases.append(("s6_slip1", 6, 0.1, rng.uniform(-1.0, 1.0, 36), [35, 3]))
    cases.append(("s5_empty", 5, 0.2, np.ones(25), []))
    names = []
    for name, size, p_slip, r, term in cases:
        P = W.IcyGridWorld(size, p_slip).p_transition
        n = size * size
        p0 = np.zeros(n)
        p0[0] = 0.5
        p0[rng.integers(0, n)] += 0.25
        p0[rng.integers(0, n)] += 0.25
        with np.errstate(all="ignore"):
            pi = M.local_action_probabilities(P, term, r)
            svf, k = ref_forward(P, p0, term, pi)
        out[f"{name}__size"] = size
        out[f"{name}__p_slip"] = p_slip
        out[f"{name}__reward"] = r
        out[f"{name}__terminal"] = np.array(term, dtype=np.int64)
        out[f"{name}__p0"] = p0
        out[f"{name}__pi"] = pi
        out[f"{name}__svf"] = svf
        out[f"{name}__k_f"] = k
        names.append(name)
        print(f"maxent_small {name}: k_f={k} finite={np.isfinite(svf).all()}")
    out["names"] = np.array(names)
    save("maxent_small", **out)


def gen_causal_small():
    """G3: soft VI + forward (causal) at 5x5, 16x16 and 32x32."""
    out = {}
    names = []
    rng = np.random.default_rng(5)
    cases = [("s5_ones", 5, np.ones(25), 0.7), ("s5_unif", 5, rng.uniform(0, 1.5, 25), 0.9),
             ("s16_unif", 16, rng.uniform(0, 1.5, 256), 0.7),
             ("s32_unif", 32, rng.uniform(0, 1.5, 1024), 0.7)]
    for name, size, r, gamma in cases:
        n = size * size
        P = W.IcyGridWorld(size, 0.2).p_transition
        term = [n - 1]
        p0 = np.zeros(n)
        p0[0] = 1.0
        t0 = time.time()
        pi, k_s = ref_soft(P, term, r, gamma)
        svf, k_f = ref_forward(P, p0, term, pi)
        out.update({f"{name}__size": size, f"{name}__reward": r, f"{name}__discount": gamma,
                    f"{name}__terminal": np.array(term), f"{name}__p0": p0, f"{name}__pi": pi,
                    f"{name}__k_s": k_s, f"{name}__svf": svf, f"{name}__k_f": k_f})
        names.append(name)
        print(f"causal_small {name}: k_s={k_s} k_f={k_f} {time.time() - t0:.1f}s")
    # terminal given as a full phi vector (maxent.py:313-314), soft pass only
    n = 25
    P = W.IcyGridWorld(5, 0.2).p_transition
    phi = np.full(n, -50.0)
    phi[24] = 0.0
    phi[4] = -1.0
    pi, k_s = ref_soft(P, phi, np.ones(n), 0.8)
    out.update({"phi_vec__phi": phi, "phi_vec__pi": pi, "phi_vec__k_s": k_s})
    out["names"] = np.array(names)
    save("causal_small", **out)


def gen_worlds():
    """G5: transition tables of the reference's world builders."""
    out = {}
    for size, p_slip in ((5, 0.2), (8, 0.1), (8, 0.3), (3, 0.2)):
        out[f"icy_{size}_{p_slip}"] = W.IcyGridWorld(size, p_slip).p_transition
    out["det_5"] = W.GridWorld(5).p_transition
    for size in (16,):
        out[f"icy_{size}_0.2_sha256"] = np.array(
            hashlib.sha256(np.ascontiguousarray(W.IcyGridWorld(size, 0.2).p_transition).tobytes()).hexdigest())
        out[f"det_{size}_sha256"] = np.array(
            hashlib.sha256(np.ascontiguousarray(W.GridWorld(size).p_transition).tobytes()).hexdigest())
    world = W.IcyGridWorld(5, 0.2)
    out["coord_features_5"] = W.coordinate_features(world)
    save("worlds", **out)


def gen_vi():
    """G6: value iteration (max and average) and policy extraction."""
    out = {}
    names = []
    rng = np.random.default_rng(6)
    for size in (5, 16):
        world = W.IcyGridWorld(size, 0.2)
        n = size * size
        r = rng.uniform(-0.5, 1.0, n)
        r[n - 1] = 2.0
        for gamma in (0.7, 0.9):
            for avg in (False, True):
                name = f"s{size}_g{int(gamma * 10)}_{'avg' if avg else 'max'}"
                v, k = ref_vi(world.p_transition, r, gamma, average=avg)
                out.update({f"{name}__size": size, f"{name}__reward": r,
                            f"{name}__discount": gamma, f"{name}__average": avg,
                            f"{name}__value": v, f"{name}__k": k})
                if not avg:
                    out[f"{name}__opt_policy"] = S.optimal_policy_from_value(world, v)
                    out[f"{name}__stoch_policy"] = S.stochastic_policy_from_value(
                        world, v, w=lambda x: np.exp(x))
                names.append(name)
                print(f"vi {name}: k={k}")
    # deterministic gridworld with ties (first-index argmax)
    world = W.GridWorld(4)
    r = np.zeros(16)
    r[15] = 1.0
    v, k = ref_vi(world.p_transition, r, 0.5)
    out.update({"det4__reward": r, "det4__value": v, "det4__k": k,
                "det4__opt_policy": S.optimal_policy_from_value(world, v)})
    out["names"] = np.array(names)
    save("vi", **out)


def random_mdp(rng, n, na, max_nnz):
    P = np.zeros((n, n, na))
    for s in range(n):
        for a in range(na):
            k = int(rng.integers(1, max_nnz + 1))
            tgt = rng.choice(n, size=k, replace=False)
            w = rng.uniform(0.1, 1.0, k)
            P[s, tgt, a] = w / w.sum()
    return P


def gen_generic():
    """G7: non-grid MDPs (generic sparse and fully dense) through every hot function."""
    rng = np.random.default_rng(7)
    out = {}
    names = []
    for name, n, na, nnz in (("sparse20", 20, 3, 6), ("dense12", 12, 2, 12), ("wide40", 40, 5, 3)):
        P = random_mdp(rng, n, na, nnz)
        r = rng.uniform(-0.3, 0.6, n)
        term = [n - 1, 2]
        p0 = rng.uniform(0, 1, n)
        p0 /= p0.sum()
        pi = M.local_action_probabilities(P, term, r)
        svf, k_f = ref_forward(P, p0, term, pi)
        cpi, k_s = ref_soft(P, term, r, 0.8)
        csvf, k_cf = ref_forward(P, p0, term, cpi)
        v, k_v = ref_vi(P, r, 0.9)
        va, k_va = ref_vi(P, r, 0.9, average=True)
        out.update({f"{name}__P": P, f"{name}__reward": r, f"{name}__terminal": np.array(term),
                    f"{name}__p0": p0, f"{name}__pi": pi, f"{name}__svf": svf, f"{name}__k_f": k_f,
                    f"{name}__cpi": cpi, f"{name}__k_s": k_s, f"{name}__csvf": csvf,
                    f"{name}__k_cf": k_cf, f"{name}__v": v, f"{name}__k_v": k_v,
                    f"{name}__va": va, f"{name}__k_va": k_va})
        names.append(name)
        print(f"generic {name}: k_f={k_f} k_s={k_s} k_cf={k_cf} k_v={k_v} k_va={k_va}")
    out["names"] = np.array(names)
    save("generic", **out)


def gen_causal_128():
    """G4 (heavy, ~20 GB RAM): reference soft VI at 128x128 in fp64 (config 5).

    The dense table is built by the oracle's vectorised builder, which the
    worlds fixture pins bit-identical to the reference builder (the reference's
    own builder needs ~10 minutes of Python calls at this size).
    """
    size = 128
    n = size * size
    rng = np.random.default_rng(5)
    theta = rng.uniform(0.0, 1.5, n)
    P = ORC.icy_gridworld_table(size, 0.2)
    chk = W.IcyGridWorld(8, 0.2).p_transition
    assert np.array_equal(chk, ORC.icy_gridworld_table(8, 0.2))
    t0 = time.time()
    pi, k_s = ref_soft(P, [n - 1], theta, 0.7)
    print(f"causal_128: k_s={k_s} {time.time() - t0:.1f}s")
    save("causal_128", theta=theta, pi=pi, k_s=k_s, size=size, discount=0.7)


class Counting:
    """Wraps a reference optimizer and counts its steps (outer IRL iterations)."""

    def __init__(self, opt):
        self.opt, self.n_steps = opt, 0

    def reset(self, parameters):
        self.opt.reset(parameters)

    def step(self, grad, *args, **kwargs):
        self.n_steps += 1
        return self.opt.step(grad, *args, **kwargs)


# the reference's other optimizers, schedules and initialisers (optimizer.py:61-108,
# 110-167, 170-214, 217-293, 334-398) on config 1's world and demonstrations
OPT_CASES = {
    "sga_power": (lambda: O.Sga(lr=O.power_decay(lr0=0.2, power=2)), lambda: O.Constant(1.0), False),
    "sga_linear": (lambda: O.Sga(lr=O.linear_decay(lr0=0.2)), lambda: O.Constant(1.0), False),
    "expsga_expdecay": (lambda: O.ExpSga(lr=O.exponential_decay(lr0=0.2, decay_rate=0.01)),
                        lambda: O.Constant(1.0), False),
    "norm_expsga": (lambda: O.ExpSga(lr=O.linear_decay(lr0=0.2)).normalize_grad(), lambda: O.Constant(1.0), False),
    "norm1_sga": (lambda: O.NormalizeGrad(O.Sga(lr=O.power_decay(lr0=0.5, decay_steps=2, power=1.5)), ord=1),
                  lambda: O.Constant(1.0), False),
    "expsga_normalize_uniform": (lambda: O.ExpSga(lr=O.linear_decay(lr0=0.2), normalize=True),
                                 lambda: O.Uniform(0.5, 1.5), False),
    "causal_norm1_sga": (lambda: O.NormalizeGrad(O.Sga(lr=O.power_decay(lr0=0.5, decay_steps=2, power=1.5)),
                                                 ord=1), lambda: O.Constant(1.0), True),
}


def gen_optimizers():
    """G7: full irl / irl_causal runs with the reference's other optimizers
    (Sga, NormalizeGrad, ExpSga(normalize), power / exponential decay, Uniform
    init seeded with np.random.seed(7)) on config 1's world and demonstrations."""
    world = W.IcyGridWorld(size=5, p_slip=0.2)
    z = np.load(os.path.join(OUT, "config1.npz"))
    flat, lens = z["traj_flat"], z["traj_lens"]
    tjs, o = [], 0
    for n in lens:
        tjs.append(T.Trajectory([tuple(int(v) for v in row) for row in flat[o:o + n]]))
        o += n
    features = W.state_features(world)
    out = {"names": np.array(list(OPT_CASES))}
    for name, (make_opt, make_init, causal) in OPT_CASES.items():
        np.random.seed(7)
        theta0 = make_init()(world.n_states)
        np.random.seed(7)
        opt = Counting(make_opt())
        if causal:
            r = M.irl_causal(world.p_transition, features, [24], tjs, opt, make_init(), 0.7)
        else:
            r = M.irl(world.p_transition, features, [24], tjs, opt, make_init())
        out[name + "__theta0"] = theta0
        out[name + "__reward"] = r
        out[name + "__steps"] = opt.n_steps
        print(f"optimizers: {name} {opt.n_steps} steps")
    save("optimizers", **out)


def gen_c2_64():
    """G8 (heavy, ~0.6 GB RAM, a few minutes): BASELINE config 2's world, 64x64
    IcyGridWorld (A = 4, p_slip 0.2, S = 4096), built by the reference's own
    builder, run through the reference with ONE BLAS thread (above 625 states
    numpy's multi-threaded row partition moves its own last bits, DESIGN.md
    section 2): value_iteration and stochastic_value_iteration (solver.py:9-104)
    at discounts 0.7 / 0.9 with values, sweep counts and optimal_policy_from_value
    (solver.py:107-124); local_causal_action_probabilities (maxent.py:279-341)
    with policy and sweep count.  Rewards: theta = 1 (mirror-symmetric states are
    exact ties that the last bit decides) and a seeded uniform theta."""
    from threadpoolctl import threadpool_limits
    size, p_slip = 64, 0.2
    n = size * size
    t0 = time.time()
    world = W.IcyGridWorld(size, p_slip)
    P = world.p_transition
    assert np.array_equal(P, ORC.icy_gridworld_table(size, p_slip))
    print(f"c2_64: reference table built in {time.time() - t0:.0f}s")
    rng = np.random.default_rng(64)
    rewards = {"ones": np.ones(n), "unif": rng.uniform(0.0, 1.5, n)}
    out = {"size": size, "p_slip": p_slip, "terminal": np.array([n - 1]),
           "P_sha256": np.array(hashlib.sha256(np.ascontiguousarray(P).tobytes()).hexdigest())}
    names = []
    with threadpool_limits(limits=1, user_api="blas"):
        for rname, r in rewards.items():
            out[f"{rname}__reward"] = r
            for gamma in (0.7, 0.9):
                for avg in (False, True):
                    name = f"{rname}_g{int(gamma * 10)}_{'avg' if avg else 'max'}"
                    t0 = time.time()
                    v, k = ref_vi(P, r, gamma, average=avg)
                    out.update({f"{name}__discount": gamma, f"{name}__average": avg, f"{name}__value": v,
                                f"{name}__k": k, f"{name}__opt_policy": S.optimal_policy_from_value(world, v)})
                    names.append(name)
                    print(f"c2_64 vi {name}: k={k} {time.time() - t0:.1f}s", flush=True)
            for gamma in (0.7, 0.9):
                name = f"{rname}_soft_g{int(gamma * 10)}"
                t0 = time.time()
                pi, k_s = ref_soft(P, [n - 1], r, gamma)
                out.update({f"{name}__discount": gamma, f"{name}__pi": pi, f"{name}__k_s": k_s})
                names.append(name)
                print(f"c2_64 soft {name}: k_s={k_s} {time.time() - t0:.1f}s", flush=True)
    out["names"] = np.array(names)
    save("c2_64", **out)


GENS = {"config1": gen_config1, "maxent_small": gen_maxent_small, "causal_small": gen_causal_small,
        "worlds": gen_worlds, "vi": gen_vi, "generic": gen_generic, "optimizers": gen_optimizers}
HEAVY = {"causal_128": gen_causal_128, "c2_64": gen_c2_64}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--heavy", action="store_true")
    args = ap.parse_args()
    todo = dict(GENS)
    if args.heavy:
        todo.update(HEAVY)
    for name, fn in todo.items():
        if args.only and name not in args.only:
            continue
        fn()


if __name__ == "__main__":
    main()
