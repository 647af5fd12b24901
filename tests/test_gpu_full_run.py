"""Full IRL runs to convergence (maxent.py:236-255) and converged-instance
compaction (irlmx.batch.BatchedMaxEnt.run(compact=True)).

Staggered convergence is made deterministic: instance 0's demonstration
statistics are its own expected SVF at theta0 = 1, so its first gradient is
exactly zero and it stops after one step (max|dtheta| = 0 <= eps); instance 1's
are that SVF plus a small offset, so it stops after a few steps; the others
use sampled demonstrations and run on.  A compacted run must equal the
uncompacted one bit for bit (theta, steps per instance), while running fewer
instances per step.
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


def staggered_workload(dev, size, n_inst, seed0=100, offset=1e-3):
    from irlmx import DeviceMDP, demos
    from irlmx.batch import BatchedMaxEnt
    S = size * size
    slips = np.linspace(0.05, 0.35, n_inst)
    mdp = DeviceMDP.icy_gridworld(size, slips, device=dev)
    rv = mdp.row_val.cpu().numpy()
    e_f = np.empty((n_inst, S))
    p0 = np.empty((n_inst, S))
    for b in range(n_inst):
        e_f[b], p0[b], _ = demos.sample(rv[b], size, [S - 1], 0, n=50, seed=seed0 + b, max_len=demos.safety_cap(size))
    svf0 = BatchedMaxEnt(mdp, e_f, p0, [S - 1]).step().cpu().numpy()   # SVF at theta0 = 1
    e_f[0] = svf0[0]
    e_f[1] = svf0[1] + offset
    return mdp, e_f, p0, [S - 1]


def run_both(mdp, e_f, p0, terminal, eps, max_steps):
    from irlmx.batch import BatchedMaxEnt
    out = {}
    for compact in (False, True):
        irl = BatchedMaxEnt(mdp, e_f, p0, terminal)
        widths = []
        r, k = irl.run(eps=eps, max_steps=max_steps, compact=compact,
                       on_step=lambda m: widths.append(m.working_batch))
        out[compact] = {"theta": irl.theta.cpu().numpy(), "reward": r.cpu().numpy(), "steps": k.cpu().numpy(),
                        "active": irl.active.cpu().numpy(), "widths": widths, "k": irl.k}
    return out[False], out[True]


def test_compaction_bit_identical_fused(dev):
    """16x16 (fused shape), six instances run to eps = 1e-4 (capped at 4,000
    steps): compacted == uncompacted bit for bit; instance 0 stops after one
    step, instance 1 after a few, and the working batch shrinks accordingly."""
    mdp, e_f, p0, term = staggered_workload(dev, 16, 6)
    full, comp = run_both(mdp, e_f, p0, term, 1e-4, 4000)
    assert full["k"] == comp["k"]
    assert np.array_equal(full["steps"], comp["steps"]), (full["steps"], comp["steps"])
    assert np.array_equal(full["theta"], comp["theta"])
    assert np.array_equal(full["reward"], comp["reward"])
    assert np.array_equal(full["active"], comp["active"])
    steps = comp["steps"]
    assert steps[0] == 1 and 1 < steps[1] < steps[2:].min(), steps
    # uncompacted: every step runs all six; compacted: 6 at step 1, then fewer
    assert set(full["widths"]) == {6}
    assert comp["widths"][0] == 6 and comp["widths"][1] == 5 and min(comp["widths"]) < 5


def test_prime_compaction_leaves_state_unchanged(dev):
    """BatchedMaxEnt.prime_compaction (run before bench.py's clocks start: it
    loads the code of the stop test, the compaction and the working-set update)
    runs on a scratch copy: the object's theta, step counts, activity and step
    index are untouched, and a run after it equals a run without it bit for bit."""
    from irlmx.batch import BatchedMaxEnt
    mdp, e_f, p0, term = staggered_workload(dev, 16, 6)
    plain = BatchedMaxEnt(mdp, e_f, p0, term)
    primed = BatchedMaxEnt(mdp, e_f, p0, term)
    theta0 = primed.theta.clone()
    primed.prime_compaction()
    assert torch.equal(primed.theta, theta0) and primed.k == 0 and primed._work is None
    assert bool(primed.active.all()) and int(primed.steps.sum()) == 0
    r1, k1 = plain.run(eps=1e-4, max_steps=4000)
    r2, k2 = primed.run(eps=1e-4, max_steps=4000)
    assert torch.equal(k1, k2) and torch.equal(r1, r2)


def test_compaction_bit_identical_cluster(dev):
    """128x128 (cluster shape, the bench's grid): five instances, five gradient
    steps with instances 0 and 1 stopping early; the compacted run re-plans for
    the smaller batch (fewer instances -> smaller tiles, more CUs per instance)
    and still equals the uncompacted run bit for bit."""
    from irlmx import ops
    mdp, e_f, p0, term = staggered_workload(dev, 128, 5)
    full, comp = run_both(mdp, e_f, p0, term, 1e-4, 5)
    assert np.array_equal(full["steps"], comp["steps"]), (full["steps"], comp["steps"])
    assert comp["steps"][0] == 1 and comp["steps"][1] < 5 and comp["steps"][2:].tolist() == [5, 5, 5]
    assert np.array_equal(full["theta"], comp["theta"])
    assert comp["widths"][0] == 5 and comp["widths"][-1] == 3
    # the bench's batch re-plans when compacted (irlmx_execution_plan)
    from irlmx import DeviceMDP
    big = DeviceMDP.icy_gridworld(128, np.linspace(0.1, 0.3, 64), device=dev)
    p64 = ops.execution_plan(big, "backward")
    p8 = ops.execution_plan(big.take(np.arange(8)), "backward")
    assert p64["shape"] == p8["shape"] == "cluster"
    assert p8["C"] > p64["C"] and p8["R"] < p64["R"], (p64, p8)


def test_run_matches_oracle_irl_loop(dev):
    """BatchedMaxEnt.run (compacted) against the oracle's irl loop (maxent.py:196-255)
    on 6x6 worlds with sampled demonstrations, per instance: the same step count
    and rewards within 1e-9; and the config-1 fixture (the reference's own
    375-step run) for a batch that mixes it with other instances."""
    from irlmx import DeviceMDP, demos
    from irlmx.batch import BatchedMaxEnt
    size, S = 6, 36
    slips = [0.1, 0.2, 0.3]
    mdp = DeviceMDP.icy_gridworld(size, slips, device=dev)
    rv = mdp.row_val.cpu().numpy()
    e_f = np.empty((3, S))
    p0 = np.empty((3, S))
    for b in range(3):
        e_f[b], p0[b], _ = demos.sample(rv[b], size, [S - 1], 0, n=40, seed=9 + b, max_len=demos.safety_cap(size))
    irl = BatchedMaxEnt(mdp, e_f, p0, [S - 1])
    r, k = irl.run(eps=1e-4)
    for b in range(3):
        P = O.icy_gridworld_table(size, slips[b])
        theta = np.ones(S)
        steps = 0
        delta = np.inf
        while delta > 1e-4:   # maxent.py:240-252 with ExpSga(linear_decay(0.2)), identity features
            pi = O.backward_maxent(P, [S - 1], theta, rescale=True)
            svf, _ = O.forward_svf(P, p0[b], [S - 1], pi)
            new = theta * np.exp(0.2 / (1.0 + steps) * (e_f[b] - svf))
            delta = np.max(np.abs(new - theta))
            theta = new
            steps += 1
        assert int(k[b]) == steps, (b, int(k[b]), steps)
        assert np.max(np.abs(r[b].cpu().numpy() - theta)) <= 1e-9 * np.max(np.abs(theta)), b
    z = load_golden("config1")
    mdp = DeviceMDP.icy_gridworld(5, [0.2, 0.35, 0.2], device=dev)
    e_f = np.tile(z["e_features"], (3, 1))   # instance 1: the same demonstrations on a slipperier world
    p0 = np.tile(z["p_initial"], (3, 1))
    r, k = BatchedMaxEnt(mdp, e_f, p0, [24]).run(eps=1e-4)
    for b in (0, 2):
        assert int(k[b]) == int(z["irl_steps"])
        assert np.max(np.abs(r[b].cpu().numpy() - z["reward_maxent"])) <= 1e-9


def test_batched_optimizers_match_reference(dev):
    """BatchedMaxEnt with the reference's other optimisers on the device
    (irlmx.optim: Sga, NormalizeGrad with ord None / 1, ExpSga with normalize,
    power / exponential decay, a Uniform-drawn theta0; optimizer.py:61-398)
    against the reference's own full irl / irl_causal runs
    (tests/golden/optimizers.npz): step counts identical, rewards within 1e-9;
    two instances per batch, both equal to the single reference run."""
    from irlmx import DeviceMDP
    from irlmx import optim as OP
    from irlmx.batch import BatchedMaxEnt
    z = load_golden("optimizers")
    c1 = load_golden("config1")
    make = {
        "sga_power": lambda: OP.Sga(lr=OP.power_decay(lr0=0.2, power=2)),
        "sga_linear": lambda: OP.Sga(lr=OP.linear_decay(lr0=0.2)),
        "expsga_expdecay": lambda: OP.ExpSga(lr=OP.exponential_decay(lr0=0.2, decay_rate=0.01)),
        "norm_expsga": lambda: OP.NormalizeGrad(OP.ExpSga(lr=OP.linear_decay(lr0=0.2))),
        "norm1_sga": lambda: OP.NormalizeGrad(OP.Sga(lr=OP.power_decay(lr0=0.5, decay_steps=2, power=1.5)), ord=1),
        "expsga_normalize_uniform": lambda: OP.ExpSga(lr=OP.linear_decay(lr0=0.2), normalize=True),
        "causal_norm1_sga": lambda: OP.NormalizeGrad(OP.Sga(lr=OP.power_decay(lr0=0.5, decay_steps=2, power=1.5)),
                                                     ord=1),
    }
    assert sorted(make) == sorted(str(n) for n in z["names"])
    mdp = DeviceMDP.icy_gridworld(5, [0.2, 0.2], device=dev)
    e_f = np.tile(c1["e_features"], (2, 1))
    p0 = np.tile(c1["p_initial"], (2, 1))
    for name, mk in make.items():
        causal = name.startswith("causal")
        irl = BatchedMaxEnt(mdp, e_f, p0, [24], causal=causal, discount=0.7 if causal else None,
                            theta0=z[name + "__theta0"], optimizer=mk())
        r, k = irl.run(eps=1e-4, max_steps=5000)
        assert k.tolist() == [int(z[name + "__steps"])] * 2, (name, k.tolist())
        for b in range(2):
            err = np.max(np.abs(r[b].cpu().numpy() - z[name + "__reward"]))
            assert err <= 1e-9 * max(1.0, np.max(np.abs(z[name + "__reward"]))), (name, b, err)


def test_dense_compaction_within_rounding(dev):
    """DENSE layout (irlmx/batch.py docstring): a compacted run re-plans from
    the shared-table GEMM (20 instances) down to the streaming / dense-grid
    kernels as instances stop, whose per-row summation orders differ -- the
    run agrees with the uncompacted one to 1e-9 (steps per instance equal),
    not bit for bit."""
    from irlmx import DeviceMDP, demos, ops
    from irlmx.batch import BatchedMaxEnt
    size, S, B = 6, 36, 20
    P = O.icy_gridworld_table(size, 0.2)
    grid = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    rv = grid.row_val.cpu().numpy()
    e_f = np.empty((B, S))
    p0 = np.empty((B, S))
    for b in range(B):
        e_f[b], p0[b], _ = demos.sample(rv[0], size, [S - 1], 0, n=30, seed=100 + b, max_len=demos.safety_cap(size))
    mdp = DeviceMDP.from_dense(P, device=dev, layout="dense").with_batch(B)
    assert ops.execution_plan(mdp, "backward")["shape"] == "dense-gemm"
    runs = {}
    for compact in (True, False):
        irl = BatchedMaxEnt(mdp, e_f, p0, [S - 1])
        runs[compact] = irl.run(eps=1e-4, compact=compact)
    (r1, k1), (r0, k0) = runs[True], runs[False]
    assert len(set(k0.tolist())) > 1                 # instances stop at different steps
    assert torch.equal(k1, k0), (k1.tolist(), k0.tolist())
    err = (r1 - r0).abs().max().item() / r0.abs().max().item()
    assert err <= 1e-9, err
