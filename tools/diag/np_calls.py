"""Per-call wall time of the numpy-order kernels vs the default shapes at 5x5 and 16x16 (config 1's world)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle")]
import torch
import maxent_oracle as O
from irlmx import DeviceMDP, ops

dev = torch.device("cuda", 0)
for size in (5, 16, 32):
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    tm = ops.terminal_mask([n - 1], n, device=dev)
    r = np.ones(n) * (0.3 if size > 12 else 1.0)
    p0 = np.zeros(n); p0[0] = 1.0
    phi = O.terminal_reward([n - 1], n)
    pi = ops.backward_maxent(mdp, r, tm)
    calls = {
        "backward": (lambda: ops.backward_maxent(mdp, r, tm), lambda: ops.backward_maxent_numpy_order(mdp, np.exp(r), tm)),
        "forward": (lambda: ops.forward_svf(mdp, p0, tm, pi), lambda: ops.forward_svf(mdp, p0, tm, pi, numpy_order=True)),
        "soft_vi": (lambda: ops.soft_backward(mdp, r, phi, 0.7), lambda: ops.soft_backward(mdp, r, phi, 0.7, numpy_order=True)),
        "vi": (lambda: ops.value_iteration(mdp, r, 0.7), lambda: ops.value_iteration(mdp, r, 0.7, numpy_order=True)),
    }
    for name, (fast, npo) in calls.items():
        out = []
        for fn in (fast, npo):
            fn(); torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                res = fn()
            torch.cuda.synchronize()
            out.append((time.perf_counter() - t) / 5 * 1e3)
        k = ""
        if name == "forward":
            k = f" ({int(res[1][0])} sweeps)"
        print(f"{size}x{size} {name}: default {out[0]:.3f} ms, numpy order {out[1]:.3f} ms{k}", flush=True)
