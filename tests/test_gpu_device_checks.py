"""The device bounds-check build (IRLMX_DEVICE_CHECKS=1, libirlmx_checks.so,
built beside the product library by __graft_entry__.build()).

One subprocess loads the check build (IRLMX_LIB) and runs the reference-pinned
cases through every execution shape -- fused, per sweep, cluster with small
tiles (halo exchanges, granule offsets, tile ranges), the persistent grid shape
on an ELL model, the compact-weight column quads at width 256 -- asserting the fixtures' results and no failed check; then a
model with a corrupted ELL index must raise the index bit instead of reading
out of bounds.  (sanitizers run on the host build, see
tests/test_host_sanitize.py; on the device this build is the bounds check.)
"""

import json
import os
import subprocess
import sys
import textwrap

import pytest

from conftest import ORACLE_DIR, PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

WORKER = textwrap.dedent("""
    import json, os, sys
    sys.path[:0] = [{root!r}, {pkg!r}, {oracle!r}, {tests!r}]
    import numpy as np, torch
    import maxent_oracle as O
    from conftest import load_golden
    from irlmx import _lib, DeviceMDP, ops
    lib = _lib.load()
    out = {{"enabled": int(lib.irlmx_device_checks_enabled()), "cases": [], "fail": []}}
    dev = torch.device("cuda", 0)
    SHAPES = {{"fused": {{}}, "sweep": {{"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER": "0", "IRLMX_GRID": "0"}},
              "cluster": {{"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER_R": "3", "IRLMX_CLUSTER_G": "2"}},
              "grid": {{"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER": "0"}}}}
    KEYS = ("IRLMX_FUSED_MAX_STATES", "IRLMX_CLUSTER", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G", "IRLMX_GRID")
    def use(shape):
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(SHAPES[shape])
    def rel(a, b):
        return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))
    z = load_golden("maxent_small")
    for shape in SHAPES:
        use(shape)
        for c in [str(n) for n in z["names"]]:
            if not np.isfinite(z[c + "__pi"]).all() or int(z[c + "__k_f"]) > 100000:
                continue
            size = int(z[c + "__size"]); n = size * size
            for layout in ("stencil", "ell"):
                mdp = DeviceMDP.from_dense(O.icy_gridworld_table(size, float(z[c + "__p_slip"])), device=dev,
                                           layout=layout)
                tm = ops.terminal_mask([int(t) for t in z[c + "__terminal"]], n, device=dev)
                pi = ops.backward_maxent(mdp, z[c + "__reward"], tm)
                svf, k, _ = ops.forward_svf(mdp, z[c + "__p0"], tm, pi)
                out["cases"].append([shape, c, layout, rel(pi[0].cpu().numpy(), z[c + "__pi"]),
                                     rel(svf[0].cpu().numpy(), z[c + "__svf"]), int(k[0]) == int(z[c + "__k_f"]),
                                     ops.device_check_failures()])
    use("grid")   # persistent grid shape: soft VI / VI and the ELL forward / backward at 128 x 128
    size = 128; n = size * size
    mdp = DeviceMDP.from_dense(O.icy_gridworld_table(size, 0.2), device=dev, layout="ell")
    r = np.random.default_rng(3).uniform(0.0, 1.0, n)
    ops.soft_backward(mdp, r, O.terminal_reward([n - 1], n), 0.7, max_iter=50)
    ops.value_iteration(mdp, r, 0.9, max_iter=20)
    tm = ops.terminal_mask([n - 1], n, device=dev)
    pi = ops.backward_maxent(mdp, r, tm)
    p0 = np.zeros(n); p0[0] = 1.0
    ops.forward_svf(mdp, p0, tm, pi, max_iter=200)
    out["grid"] = ops.device_check_failures()
    # width 256: the compact-weight column quads (cluster.hip LAY 4), the planner's
    # plan and a forced one at 20 states per lane, against the per-sweep shape
    size = 256; n = size * size
    mdp = DeviceMDP.icy_gridworld(size, [0.15, 0.3], device=dev)
    r = np.random.default_rng(8).uniform(-1.0, 1.0, (2, n))
    tm = ops.terminal_mask([n - 1], n, batch=2, device=dev)
    res = []
    for env in ({{}}, {{"IRLMX_CLUSTER_R": "24", "IRLMX_CLUSTER_G": "8"}}, {{"IRLMX_CLUSTER": "0"}}):
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        res.append((ops.execution_plan(mdp, "backward")["layout"], ops.backward_maxent(mdp, r, tm)))
    out["w256"] = [res[0][0], res[1][0], bool(torch.equal(res[0][1], res[2][1])),
                   bool(torch.equal(res[1][1], res[2][1])), ops.device_check_failures()]
    # a corrupted ELL index: the check bit instead of an out-of-bounds read
    use("sweep")
    g = load_golden("generic")
    mdp = DeviceMDP.from_dense(g["sparse20__P"], device=dev, layout="ell")
    mdp.row_idx[0, 1, 3] = 20 + 7
    tm = ops.terminal_mask([int(t) for t in g["sparse20__terminal"]], 20, device=dev)
    ops.backward_maxent(mdp, g["sparse20__reward"], tm)
    out["corrupt"] = ops.device_check_failures()
    out["after"] = ops.device_check_failures()
    json.dump(out, open({out!r}, "w"))
""")


def test_device_check_build(tmp_path):
    import __graft_entry__ as g
    g.build()
    res = str(tmp_path / "checks.json")
    code = WORKER.format(root=ROOT, pkg=PKG_DIR, oracle=ORACLE_DIR, tests=os.path.join(ROOT, "tests"), out=res)
    env = dict(os.environ, IRLMX_LIB=g.LIB_CHECKS)
    subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, check=True, timeout=600)
    out = json.load(open(res))
    assert out["enabled"] == 1
    assert len(out["cases"]) >= 4 * 2 * 6
    for shape, case, layout, e_pi, e_svf, same_k, fails in out["cases"]:
        assert fails == 0, (shape, case, layout, fails)
        assert e_pi <= 1e-9 and e_svf <= 1e-8 and same_k, (shape, case, layout, e_pi, e_svf, same_k)
    assert out["grid"] == 0
    assert out["w256"] == [4, 4, True, True, 0], out["w256"]
    assert out["corrupt"] & 1, out["corrupt"]   # kCheckIndex
    assert out["after"] == 0                    # cleared by the read
