"""Kernels of one config-3 forward call (128x128, B = 64) capped at K sweeps,
for rocprofv3 --kernel-trace --stats: which part of the per-call fixed cost
(tools/diag/fwd_fixed_cost.py) is the workspace memset, the weights kernel and
the persistent kernel's own prologue / epilogue."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch  # noqa: E402
from irlmx import DeviceMDP, ops  # noqa: E402

dev = torch.device("cuda", 0)
size, B, K = 128, 64, int(os.environ.get("K", 8))
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
p0 = torch.zeros((B, n), dtype=torch.float64, device=dev); p0[:, 0] = 1.0
pi = ops.backward_maxent(mdp, r, tm)
for _ in range(20):
    ops.forward_svf(mdp, p0, tm, pi, max_iter=K)
torch.cuda.synchronize()
print("done", K, flush=True)
