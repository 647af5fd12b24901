"""Dense-row path (IRLMX_LAYOUT_DENSE, csrc/dense.hip) against the oracle.

Transition models whose rows are mostly nonzero (non-grid MDPs) are kept as
per-action S x S row-major matrices and streamed one wave per row; with one
table shared by B instances every sweep's P . [v_1 .. v_B] contraction runs as
one GEMM over all instances on the hand-written fp64 MFMA kernel
(dense.hip dense_gemm_kernel; no library GEMM).  Checked here:

* the generic fixtures (tests/golden/generic.npz: reference outputs for three
  non-grid MDPs, tools/gen_golden.py), forced onto the DENSE layout;
* a seeded random dense MDP with S = 2048, A = 4 (every entry nonzero,
  oracle.random_dense_mdp) against the dense oracle's outputs
  (tests/golden/dense2048.npz, tools/gen_full_fixtures.py): backward
  (maxent.py:155), forward (:109), soft VI (:329) + causal forward, VI and its
  action average (solver.py:44, 99) -- sweep counts identical, values within
  1e-9 relative;
* the shared-table GEMM backward equals the per-instance streaming kernel to
  1e-12 and the oracle to 1e-9.
"""

import numpy as np
import pytest

import maxent_oracle as O
from conftest import load_golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CONTRACT = 1e-5


def close(got, ref, rtol, what):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    assert np.array_equal(np.isfinite(got), np.isfinite(ref)), what
    fin = np.isfinite(ref)
    err = np.max(np.abs(got[fin] - ref[fin])) / max(np.max(np.abs(ref[fin])), 1e-300)
    assert err <= CONTRACT and err <= rtol, (what, err)


@pytest.fixture(scope="module")
def dev():
    import __graft_entry__ as g
    g.build()
    import irlmx
    return irlmx.require_device()


def run_all(mdp, r, term, p0, dev):
    from irlmx import ops
    from irlmx.batch import terminal_reward
    n = mdp.n_states
    tm = ops.terminal_mask(term, n, device=dev)
    out = {"pi": ops.backward_maxent(mdp, r, tm)[0].cpu().numpy()}
    svf, k, _ = ops.forward_svf(mdp, p0, tm, out["pi"])
    out.update(svf=svf[0].cpu().numpy(), k_f=int(k[0]))
    cpi, cv, ks, _ = ops.soft_backward(mdp, r, terminal_reward(term, n, 1, dev), 0.8 if n < 100 else 0.7)
    out.update(cpi=cpi[0].cpu().numpy(), cv=cv[0].cpu().numpy(), k_s=int(ks[0]))
    csvf, kc, _ = ops.forward_svf(mdp, p0, tm, out["cpi"])
    out.update(csvf=csvf[0].cpu().numpy(), k_cf=int(kc[0]))
    v, kv, _ = ops.value_iteration(mdp, r, 0.9)
    va, kva, _ = ops.value_iteration(mdp, r, 0.9, average=True)
    out.update(v=v[0].cpu().numpy(), k_v=int(kv[0]), va=va[0].cpu().numpy(), k_va=int(kva[0]))
    return out


def test_generic_fixtures_on_dense_layout(dev):
    from irlmx import DeviceMDP, _lib, ops
    z = load_golden("generic")
    for c in [str(n) for n in z["names"]]:
        P = z[c + "__P"]
        mdp = DeviceMDP.from_dense(P, device=dev, layout="dense")
        assert mdp.layout == _lib.LAYOUT_DENSE
        # every pass on the persistent dense shape (test_gpu_dense_grid.py)
        assert ops.execution_plan(mdp, "forward")["shape"] == "dense-grid"
        assert ops.execution_plan(mdp, "soft_backward")["shape"] == "dense-grid"
        term = [int(t) for t in z[c + "__terminal"]]
        got = run_all(mdp, z[c + "__reward"], term, z[c + "__p0"], dev)
        close(got["pi"], z[c + "__pi"], 1e-9, c + " pi")
        assert got["k_f"] == int(z[c + "__k_f"]), c
        close(got["svf"], z[c + "__svf"], 1e-8, c + " svf")
        # (the generic fixtures' soft VI ran at discount 0.8)
        assert got["k_s"] == int(z[c + "__k_s"]), c
        close(got["cpi"], z[c + "__cpi"], 1e-9, c + " cpi")
        assert got["k_cf"] == int(z[c + "__k_cf"]), c
        close(got["csvf"], z[c + "__csvf"], 1e-8, c + " csvf")
        assert got["k_v"] == int(z[c + "__k_v"]) and got["k_va"] == int(z[c + "__k_va"]), c
        close(got["v"], z[c + "__v"], 1e-12, c + " v")
        close(got["va"], z[c + "__va"], 1e-12, c + " va")


@pytest.fixture(scope="module")
def dense2048():
    z = load_golden("dense2048")
    P, r, term, p0 = O.random_dense_mdp()
    assert np.array_equal(np.array([P.sum(), P[::7, ::5, :].sum(), P[-1, -1, -1]]), z["P_check"])
    assert np.array_equal(r, z["reward"])
    return P, r, term, p0, z


def test_random_dense_2048_vs_dense_oracle(dev, dense2048):
    from irlmx import DeviceMDP, _lib, ops
    P, r, term, p0, z = dense2048
    mdp = DeviceMDP.from_dense(P, device=dev)     # picked automatically: rows are full
    assert mdp.layout == _lib.LAYOUT_DENSE
    assert ops.execution_plan(mdp, "backward")["shape"] == "dense-grid"
    assert ops.execution_plan(mdp, "value_iteration")["shape"] == "dense"
    got = run_all(mdp, r, term, p0, dev)
    close(got["pi"], z["pi"], 1e-9, "pi")
    assert np.argmax(got["pi"], axis=1).tolist() == np.argmax(z["pi"], axis=1).tolist()
    for k in ("k_f", "k_s", "k_cf", "k_v", "k_va"):
        assert got[k] == int(z[k]), (k, got[k], int(z[k]))
    close(got["svf"], z["svf"], 1e-9, "svf")
    close(got["cpi"], z["cpi"], 1e-9, "cpi")
    close(got["cv"], z["cv"], 1e-9, "cv")
    close(got["csvf"], z["csvf"], 1e-9, "csvf")
    close(got["v"], z["v"], 1e-12, "v")
    close(got["va"], z["va"], 1e-12, "va")


def test_shared_table_gemm_backward(dev, dense2048, monkeypatch):
    """One dense table, 16 reward vectors: the backward sweep as one GEMM over all
    instances (plan "dense-gemm", the hand-written fp64 MFMA kernel) equals the
    per-instance streaming kernel and the oracle (instance 0 carries the
    fixture's reward)."""
    from irlmx import DeviceMDP, ops
    P, r, term, p0, z = dense2048
    B = 16
    mdp = DeviceMDP.from_dense(P, device=dev).with_batch(B)
    rew = np.random.default_rng(16).uniform(0.0, 1.0, (B, P.shape[0]))
    rew[0] = r
    tm = ops.terminal_mask(term, P.shape[0], batch=B, device=dev)
    assert ops.execution_plan(mdp, "backward")["shape"] == "dense-gemm"   # 16 instances: the MFMA kernel
    pi_gemm = ops.backward_maxent(mdp, rew, tm).cpu().numpy()            # hand-written fp64 MFMA kernel
    monkeypatch.setenv("IRLMX_DENSE_GEMM_MIN", "1000000")
    assert ops.execution_plan(mdp, "backward")["shape"] == "dense"
    pi_stream = ops.backward_maxent(mdp, rew, tm).cpu().numpy()
    close(pi_gemm, pi_stream, 1e-12, "gemm vs streaming")
    close(pi_gemm[0], z["pi"], 1e-9, "gemm vs oracle")


def test_dropin_accepts_dense_tables(dev, dense2048):
    """The numpy drop-ins (maxent.py / solver.py) route a dense ndarray to the
    DENSE layout; results as the oracle's."""
    import maxent as M
    import solver as S
    P, r, term, p0, z = dense2048
    close(M.local_action_probabilities(P, term, r), z["pi"], 1e-9, "drop-in pi")
    close(S.value_iteration(P, r, 0.9), z["v"], 1e-12, "drop-in v")


@pytest.mark.parametrize("n,batch", [(300, 5), (301, 3), (302, 17), (1040, 37), (1037, 20)])
def test_gemm_edges(dev, monkeypatch, n, batch):
    """The MFMA kernel's partial row / instance tiles (S not a multiple of 32, B not
    a multiple of 16) and its K tail (S % 4 != 0, odd S: element-wise loads)
    against the streaming kernel, forced onto the GEMM plan."""
    from irlmx import DeviceMDP, ops
    P, _, _, _ = O.random_dense_mdp(n, 3, seed=n)
    mdp = DeviceMDP.from_dense(P, device=dev, layout="dense").with_batch(batch)
    rew = np.random.default_rng(n).uniform(0.0, 1.0, (batch, n))
    tm = ops.terminal_mask([n - 1], n, batch=batch, device=dev)
    monkeypatch.setenv("IRLMX_DENSE_GEMM_MIN", "2")
    assert ops.execution_plan(mdp, "backward")["shape"] == "dense-gemm"
    pi_gemm = ops.backward_maxent(mdp, rew, tm).cpu().numpy()
    monkeypatch.setenv("IRLMX_DENSE_GEMM_MIN", "1000000")
    pi_stream = ops.backward_maxent(mdp, rew, tm).cpu().numpy()
    close(pi_gemm, pi_stream, 1e-12, f"gemm vs streaming S={n} B={batch}")


def test_shared_table_gemm_soft_vi_and_vi(dev, dense2048, monkeypatch):
    """Soft VI (maxent.py:326-338) and VI (solver.py:40-50) of 16 reward vectors on one
    dense table: every sweep's P_a . [v_1 .. v_16] on the fp64 MFMA kernel (plan
    "dense-gemm"), against the per-instance streaming kernel (sweep counts
    identical, values within 1e-12) and the dense oracle (instance 0)."""
    from irlmx import DeviceMDP, ops
    from irlmx.batch import terminal_reward
    P, r, term, p0, z = dense2048
    n, B = P.shape[0], 16
    mdp = DeviceMDP.from_dense(P, device=dev).with_batch(B)
    rew = np.random.default_rng(161).uniform(0.0, 1.0, (B, n))
    rew[0] = r
    phi = terminal_reward(term, n, B, dev)
    assert ops.execution_plan(mdp, "soft_backward")["shape"] == "dense-gemm"

    def run():
        cpi, cv, ks, _ = ops.soft_backward(mdp, rew, phi, 0.7)
        v, kv, _ = ops.value_iteration(mdp, rew, 0.9)
        return cpi.cpu().numpy(), cv.cpu().numpy(), ks.cpu().numpy(), v.cpu().numpy(), kv.cpu().numpy()

    g = run()
    monkeypatch.setenv("IRLMX_DENSE_GEMM_MIN", "1000000")
    assert ops.execution_plan(mdp, "soft_backward")["shape"] == "dense"
    s = run()
    assert np.array_equal(g[2], s[2]) and np.array_equal(g[4], s[4])
    for i in (0, 1, 3):
        close(g[i], s[i], 1e-12, f"gemm vs streaming {i}")
    assert int(g[2][0]) == int(z["k_s"]) and int(g[4][0]) == int(z["k_v"])
    close(g[0][0], z["cpi"], 1e-9, "soft pi vs oracle")
    close(g[3][0], z["v"], 1e-12, "v vs oracle")


# (rows, n, batch, expected variant): every kernel variant dense_gemm_launch picks,
# with partial tiles and K tails: {row tiles, instance tiles, waves, 16-byte loads}
GEMM_SHAPES = [
    (300, 300, 5, (1, 1, 8, 1)), (301, 301, 3, (1, 1, 8, 0)), (1040, 1037, 20, (1, 1, 8, 0)),
    (4096, 4096, 16, (1, 1, 8, 1)), (4096, 4096, 64, (2, 2, 8, 1)), (8192, 4094, 16, (2, 1, 8, 1)),
    (16384, 2049, 16, (2, 1, 4, 0)), (8192, 8192, 64, (2, 4, 8, 1)), (16384, 1030, 33, (2, 2, 4, 1)),
    (2048 * 4, 2048, 16, (2, 1, 8, 1)), (2048, 2048, 64, (2, 1, 8, 1)), (4096, 4096, 32, (2, 1, 8, 1)),
]


@pytest.mark.parametrize("rows,n,batch,variant", GEMM_SHAPES)
def test_dense_gemm_kernel_vs_torch(dev, rows, n, batch, variant):
    """irlmx_dense_gemm (C = Z . M^T on v_mfma_f64_16x16x4_f64) against torch's
    fp64 matmul of the same operands, for every variant of the kernel -- the
    8-wave ST = 2 / NBT = 4 form with 128 KiB of LDS at S = 8192, B = 64 included
    -- and K tails (n % 16 != 0, odd n); relative error within 1e-13."""
    from irlmx import ops
    assert ops.dense_gemm_variant(rows, n, batch) == variant
    g = torch.Generator(device=dev).manual_seed(rows + n + batch)
    m = torch.rand((rows, n), dtype=torch.float64, device=dev, generator=g)
    z = torch.rand((batch, n), dtype=torch.float64, device=dev, generator=g)
    c = ops.dense_gemm(m, z)
    ref = z @ m.T
    err = float((c - ref).abs().max() / ref.abs().max())
    assert err <= 1e-13, (rows, n, batch, err)
    # deterministic: a second call is bit-identical
    assert torch.equal(ops.dense_gemm(m, z), c)


def test_dense_8192_shared_table(dev):
    """A dense S = 8192 table (2.1 GB of rows) shared by 64 instances: the VI
    sweep (solver.py:40-50) on the GEMM plan (the stacked [4 S x S] products,
    LDS-staged epilogue vectors) for a capped number of sweeps, against the
    per-instance streaming kernel; also the LDS-staged streaming kernels at
    S = 8192 with B > 1 (64 KiB of dynamic LDS)."""
    from irlmx import DeviceMDP, ops
    n, B = 8192, 64
    P, _, _, _ = O.random_dense_mdp(n, 4, seed=8192)
    mdp = DeviceMDP.from_dense(P, device=dev, layout="dense").with_batch(B)
    del P
    rew = np.random.default_rng(8192).uniform(0.0, 1.0, (B, n))
    assert ops.execution_plan(mdp, "value_iteration")["shape"] == "dense-gemm"
    v_g, k_g, st_g = ops.value_iteration(mdp, rew, 0.9, max_iter=6)
    import os
    os.environ["IRLMX_DENSE_GEMM_MIN"] = "1000000"
    try:
        assert ops.execution_plan(mdp, "value_iteration")["shape"] == "dense"
        v_s, k_s, st_s = ops.value_iteration(mdp, rew, 0.9, max_iter=6)
    finally:
        del os.environ["IRLMX_DENSE_GEMM_MIN"]
    assert k_g.tolist() == k_s.tolist() == [6] * B
    close(v_g.cpu().numpy(), v_s.cpu().numpy(), 1e-12, "S=8192 VI gemm vs streaming")
    torch.cuda.synchronize()
