"""Compare forward/backward results of the fused, sweep and cluster shapes bit for bit."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle")]
import torch
from irlmx import DeviceMDP, ops

SHAPES = {"fused": {}, "sweep": {"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER": "0"},
          "cluster": {"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER_R": "3", "IRLMX_CLUSTER_G": "2"}}
dev = torch.device("cuda", 0)
rng = np.random.default_rng(3)
for size, theta, maxit in ((8, "ones", 0), (8, "unif", 20000), (12, "ones", 0)):
    n = size * size
    r = np.ones(n) if theta == "ones" else rng.uniform(0, 1.5, n)
    p0 = np.zeros(n); p0[0] = 1.0
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    tm = ops.terminal_mask([n - 1], n, device=dev)
    res = {}
    for name, env in SHAPES.items():
        for k in ("IRLMX_FUSED_MAX_STATES", "IRLMX_CLUSTER", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
            os.environ.pop(k, None)
        os.environ.update(env)
        pi = ops.backward_maxent(mdp, r, tm)
        svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=maxit)
        res[name] = (pi[0].cpu().numpy(), svf[0].cpu().numpy(), int(k[0]))
    for name in ("sweep", "cluster"):
        a, b = res["fused"], res[name]
        dpi = np.max(np.abs(a[0] - b[0]))
        dsv = np.max(np.abs(a[1] - b[1]))
        print(f"{size}x{size} {theta}: {name:7s} pi bitwise={np.array_equal(a[0], b[0])} (max {dpi:.3e}) "
              f"svf bitwise={np.array_equal(a[1], b[1])} (max {dsv:.3e}) k={a[2]} vs {b[2]}")
