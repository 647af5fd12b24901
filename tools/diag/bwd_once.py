"""One warm-up and one measured backward pass at config 3 (128x128, B = 64), for
rocprofv3 counter passes on the cluster kernel."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size, B = 128, 64
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
for _ in range(2):
    ops.backward_maxent(mdp, r, tm)
torch.cuda.synchronize()
print("done")
