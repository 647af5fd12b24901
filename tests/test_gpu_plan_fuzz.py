"""Seeded random tile plans of the cluster kernels against the per-sweep shape.

The parity tests pin the planner's own plans and a few forced small ones; this
draws 32 cases from a fixed seed -- grid width and height (square and
rectangular, widths with compile-time LDS offsets and generic ones), batch,
in-tile layout (IRLMX_PAIR), forced owned rows R and ghost rows G (ghosts wider
than tiles included), rewards of both signs, terminals, initial distributions
and forward caps -- and requires the cluster shape's policy, SVF, sweep counts
and status to equal the per-sweep shape's bit for bit (both compute the same
float64 operations in the same order: cluster.hip).  Cases whose forced plan
does not fit a CU fall back to the planner's own plan (still compared); at
least half of the (case, pass) pairs must run the forced cluster plan.
"""

import numpy as np
import pytest

from conftest import icy_stencil_rect

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N_CASES = 32
KEYS = ("IRLMX_FUSED_MAX_STATES", "IRLMX_CLUSTER", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G", "IRLMX_PAIR",
        "IRLMX_GRID", "IRLMX_COMPACT")


@pytest.fixture(scope="module")
def dev():
    import __graft_entry__ as g
    g.build()
    import irlmx
    return irlmx.require_device()


def draw(rng):
    W = int(rng.choice([16, 24, 37, 64, 128, 256]))
    H = int(W if rng.random() < 0.5 else rng.integers(4, max(5, min(2 * W, 65536 // W))))
    B = int(rng.integers(1, 5))
    layouts = {64: [-1, 0, 1, 2], 128: [-1, 0, 1, 2, 3], 256: [-1, 0, 3, 4]}.get(W, [-1])
    # rows one CU's registers hold at the smallest states-per-lane budget of the
    # width's layouts (cluster.hip cluster_plan): forced plans mostly fit
    rows = {64: 96, 128: 48, 256: 24}.get(W, 6144 // W)
    G = int(rng.integers(1, min(16, max(1, rows // 2 - 1)) + 1))
    R = int(rng.integers(1, max(1, min(H, rows - 2 * G)) + 1))
    return dict(W=W, H=H, B=B, layout=int(rng.choice(layouts)), R=R, G=G,
                # (random rewards can keep the forward from converging for
                # millions of sweeps: every case has a cap)
                cap=int(rng.choice([1, 7, 500, 3000, 20000])) if W * H > 4096 else 50000,
                neg=bool(rng.random() < 0.5), seed=int(rng.integers(1 << 30)))


def set_env(monkeypatch, env):
    for k in KEYS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))


def test_random_cluster_plans_bit_identical(dev, monkeypatch):
    from irlmx import DeviceMDP, _lib, ops
    rng = np.random.default_rng(20261018)
    forced = 0
    for i in range(N_CASES):
        c = draw(rng)
        W, H, B = c["W"], c["H"], c["B"]
        S = W * H
        r_ = np.random.default_rng(c["seed"])
        slips = r_.uniform(0.05, 0.4, B)
        if W == H and r_.random() < 0.5:
            mdp = DeviceMDP.icy_gridworld(W, slips, device=dev)
        else:
            rv = np.stack([icy_stencil_rect(W, H, p) for p in slips])
            mdp = DeviceMDP(_lib.LAYOUT_STENCIL5, S, 4, B, False, torch.as_tensor(rv, device=dev), width=W,
                            height=H, device=dev)
        lo = -1.0 if c["neg"] else 0.0
        reward = r_.uniform(lo, 1.5, (B, S))
        terminal = sorted(set([S - 1] + [int(t) for t in r_.integers(0, S, int(r_.integers(0, 3)))]))
        tm = ops.terminal_mask(terminal, S, batch=B, device=dev)
        p0 = r_.random((B, S)) ** 8
        p0 /= p0.sum(axis=1, keepdims=True)
        env = {"IRLMX_FUSED_MAX_STATES": 0, "IRLMX_CLUSTER_R": c["R"], "IRLMX_CLUSTER_G": c["G"]}
        if c["layout"] >= 0:
            env["IRLMX_PAIR"] = c["layout"]
        out = {}
        for name, e in (("cluster", env), ("sweep", {"IRLMX_FUSED_MAX_STATES": 0, "IRLMX_CLUSTER": 0})):
            set_env(monkeypatch, e)
            plans = [ops.execution_plan(mdp, op) for op in ("backward", "forward")]
            pi = ops.backward_maxent(mdp, reward, tm)
            svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=c["cap"])
            out[name] = (plans, pi, svf, k, st)
        set_env(monkeypatch, {})
        plans = out["cluster"][0]
        hit = [p["shape"] == "cluster" and p["R"] == c["R"] and p["G"] == c["G"] for p in plans]
        forced += sum(hit)
        print(f"[fuzz {i}] {c} plans {[(p['shape'], p['R'], p['G'], p['C'], p['spt'], p['layout']) for p in plans]} "
              f"k_f {out['sweep'][3].tolist()}", flush=True)
        a, b = out["sweep"], out["cluster"]
        assert torch.equal(a[1], b[1]), (i, c, "pi")
        assert torch.equal(a[3], b[3]) and torch.equal(a[4], b[4]), (i, c, a[3].tolist(), b[3].tolist())
        fin = torch.isfinite(a[2])
        assert torch.equal(fin, torch.isfinite(b[2])) and torch.equal(a[2][fin], b[2][fin]), (i, c, "svf")
    assert forced >= 2 * N_CASES // 2, forced


def test_random_soft_vi_and_vi_bit_identical(dev, monkeypatch):
    """Soft VI (maxent.py:326-338) and value iteration (solver.py:40-50, 95-100)
    on 16 seeded random grids (square and rectangular, batch 1-5, discounts
    0.5-0.95, rewards of both signs, extra terminals) through the shape the
    library picks (fused, or the persistent grid shape above 4,096 states)
    against the per-sweep shape: values, policies, sweep counts and status bit
    for bit."""
    from irlmx import DeviceMDP, _lib, ops
    from irlmx.batch import terminal_reward
    rng = np.random.default_rng(181026)
    shapes = set()
    for i in range(16):
        W = int(rng.choice([16, 37, 64, 128, 200, 256]))
        H = int(W if rng.random() < 0.5 else rng.integers(4, max(5, min(2 * W, 65536 // W))))
        B, S = int(rng.integers(1, 6)), W * H
        gamma = float(rng.choice([0.5, 0.7, 0.9, 0.95]))
        slips = rng.uniform(0.05, 0.4, B)
        rv = np.stack([icy_stencil_rect(W, H, p) for p in slips])
        mdp = DeviceMDP(_lib.LAYOUT_STENCIL5, S, 4, B, False, torch.as_tensor(rv, device=dev), width=W, height=H,
                        device=dev)
        r = rng.uniform(-1.0 if rng.random() < 0.5 else 0.0, 1.5, (B, S))
        phi = terminal_reward(sorted(set([S - 1] + [int(t) for t in rng.integers(0, S, 2)])), S, B, dev)
        out = {}
        for name, env in (("default", {}), ("sweep", {"IRLMX_FUSED_MAX_STATES": 0, "IRLMX_GRID": 0})):
            set_env(monkeypatch, env)
            shape = ops.execution_plan(mdp, "soft_backward")["shape"]
            out[name] = (ops.soft_backward(mdp, r, phi, gamma, max_iter=20000), ops.value_iteration(mdp, r, gamma),
                         ops.value_iteration(mdp, r, gamma, average=True))
            if name == "default":
                shapes.add(shape)
                case_shape = shape
        set_env(monkeypatch, {})
        print(f"[fuzz vi {i}] W={W} H={H} B={B} gamma={gamma} shape={case_shape} "
              f"k_soft={out['sweep'][0][2].tolist()} k_vi={out['sweep'][1][1].tolist()}", flush=True)
        for got, ref in zip(out["default"], out["sweep"]):
            for x, y in zip(got, ref):
                assert torch.equal(x.view(torch.int64) if x.dtype == torch.float64 else x,
                                   y.view(torch.int64) if y.dtype == torch.float64 else y), (i, W, H, B, gamma)
    assert "grid" in shapes, shapes


def stencil_csr(rv, W, H):
    """Per-action CSR matrices P_a[from, to] of a STENCIL5 row table [A, 5, S]
    (slot 0: self, slots 1-4: the neighbours (+x, -x, +y, -y))."""
    import scipy.sparse as sp
    S = W * H
    s = np.arange(S)
    off = [0, 1, -1, W, -W]
    mats = []
    for a in range(rv.shape[0]):
        rows, cols, vals = [], [], []
        for k in range(5):
            nz = rv[a, k] != 0.0
            rows.append(s[nz])
            cols.append(s[nz] + off[k])
            vals.append(rv[a, k][nz])
        mats.append(sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(S, S)))
    return mats


def test_random_rectangular_grids_against_oracle(dev, monkeypatch):
    """Eight seeded rectangular grids (up to ~2,000 states) through the library's
    default shapes and a forced cluster plan, against the CPU oracle's CSR
    restatement of the reference (oracle/maxent_oracle.py: backward
    maxent.py:119-159, forward maxent.py:63-114, soft VI maxent.py:279-341):
    sweep counts identical, policies / SVF / values within 1e-9 relative."""
    import maxent_oracle as O
    from irlmx import DeviceMDP, _lib, ops
    from irlmx.batch import terminal_reward
    rng = np.random.default_rng(1810)
    for i in range(8):
        W = int(rng.integers(3, 60))
        H = int(rng.integers(3, max(4, min(60, 2000 // W))))
        S = W * H
        slip = float(rng.uniform(0.05, 0.4))
        rv = icy_stencil_rect(W, H, slip)
        mats = stencil_csr(rv, W, H)
        terminal = sorted(set([S - 1] + [int(t) for t in rng.integers(0, S, int(rng.integers(0, 3)))]))
        reward = rng.uniform(-0.5, 1.0, S)
        if i % 2 == 0:
            reward[terminal] = 4.0   # a policy drawn to the terminals: the forward converges (~100-250 sweeps)
        p0 = rng.random(S) ** 8
        p0 /= p0.sum()
        gamma = float(rng.choice([0.5, 0.7, 0.9]))
        pi_ref = O.backward_maxent_csr(mats, terminal, reward)
        svf_ref, k_ref = O.forward_svf_csr(mats, p0, terminal, pi_ref, max_iter=20000)
        spi_ref, v_ref, ks_ref = O.soft_backward_csr(mats, terminal, reward, gamma)
        mdp = DeviceMDP(_lib.LAYOUT_STENCIL5, S, 4, 1, False, torch.as_tensor(rv[None], device=dev), width=W,
                        height=H, device=dev)
        tm = ops.terminal_mask(terminal, S, device=dev)
        phi = terminal_reward(terminal, S, 1, dev)
        for name, env in (("default", {}), ("cluster", {"IRLMX_FUSED_MAX_STATES": 0, "IRLMX_CLUSTER_R": 2,
                                                        "IRLMX_CLUSTER_G": int(rng.integers(1, 9))})):
            set_env(monkeypatch, env)
            pi = ops.backward_maxent(mdp, reward, tm)
            svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=20000)
            spi, v, ks, _ = ops.soft_backward(mdp, reward, phi, gamma)
            what = (i, W, H, name, ops.execution_plan(mdp, "forward")["shape"])
            print(f"[oracle {i}] W={W} H={H} {name} shape={what[-1]} k_f={int(k[0])} (oracle {k_ref}) "
                  f"k_soft={int(ks[0])} (oracle {ks_ref})", flush=True)
            assert int(k[0]) == k_ref and int(ks[0]) == ks_ref, what
            for got, ref in ((pi[0], pi_ref), (svf[0], svf_ref), (spi[0], spi_ref), (v[0], v_ref)):
                got = got.cpu().numpy()
                fin = np.isfinite(ref)
                assert np.array_equal(fin, np.isfinite(got)), what
                e = np.max(np.abs(got[fin] - ref[fin])) / np.max(np.abs(ref[fin]))
                assert e <= 1e-9, (what, e)
        set_env(monkeypatch, {})
